// pybind11 entry points of the _pra_hip kernel library. Arguments are raw device
// pointers (ints from torch.Tensor.data_ptr()) and the current HIP stream, so the
// Python side pays one pybind11 call per launch and no tensor marshalling.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <vector>
#include <stdint.h>
#include <stdexcept>
#include <string>

namespace py = pybind11;
typedef uintptr_t P;

extern "C" {
void pra_layernorm_fwd(const void*, const void*, const void*, void*, float*, float*, int, int, float, int, int,
                       hipStream_t);
void pra_layernorm_bwd(const void*, const void*, const void*, const float*, const float*, void*, float*, float*, int,
                       int, int, int, int, hipStream_t);
void pra_rmsnorm_fwd(const void*, const void*, void*, float*, int, int, float, int, int, hipStream_t);
void pra_rmsnorm_bwd(const void*, const void*, const void*, const float*, void*, float*, int, int, int, int, int,
                     hipStream_t);
void pra_colsum(const float*, void*, int, int, int, hipStream_t);
void pra_softmax_fwd(const void*, void*, int, int, int, hipStream_t);
void pra_softmax_bwd(const void*, const void*, void*, int, int, int, hipStream_t);
void pra_softmax_ce_fwd(const void*, const int64_t*, float*, float*, int, int, int, int, hipStream_t);
void pra_softmax_ce_bwd(const void*, const int64_t*, const float*, const float*, void*, int, int, int, int,
                        hipStream_t);
void pra_vp_ce_part_fwd(const void*, const int64_t*, float*, int, int, int64_t, int, hipStream_t);
void pra_vp_ce_final(const float*, const int64_t*, float*, float*, int, int, int64_t, int, hipStream_t);
void pra_vp_ce_bwd(const void*, const int64_t*, const float*, const float*, void*, int, int, int64_t, int64_t, int,
                   int, hipStream_t);
const char* pra_build_info();
int pra_mmha_splits(int, int, int);
int pra_mmha_decode(const void*, void*, const float*, float*, void*, int, int, int, int, int, const int*, int, int,
                    float, int, hipStream_t);
void pra_bias_gelu_fwd(const void*, const void*, void*, int64_t, int, int, int, hipStream_t);
void pra_bias_gelu_bwd(const void*, const void*, const void*, void*, int64_t, int, int, int, hipStream_t);
void pra_adamw_mt(const int64_t*, const float*, const int64_t*, int, float, float, float, float, float, float, float,
                  const float*, hipStream_t);
void pra_lamb_shard_stage1(const int64_t*, int, const void*, int, const float*, float*, float*, float*, const float*,
                           float*, int, float, float, float, float, float, float, const float*, hipStream_t);
void pra_lamb_shard_stage2(const int64_t*, int, float*, const float*, const float*, int, float, void*, int,
                           hipStream_t);
void pra_zero_mt(const int64_t*, int, hipStream_t);
void pra_momentum_mt(const int64_t*, const float*, const int64_t*, int, float, float, int, float, const float*,
                     hipStream_t);
void pra_sumsq_accum(const void*, float*, int64_t, int, hipStream_t);
void pra_flash_bwd_pre(const void*, const void*, float*, int, int, int, int, int, hipStream_t);
int pra_adl_supported(int);
void pra_adl_fwd(const void*, const void*, const void*, const void*, const void*, void*, void*, float*, float*, int,
                 int, float, float, uint64_t, uint64_t, const uint64_t*, int, int, hipStream_t);
void pra_adl_bwd(const void*, const void*, const void*, const void*, const float*, const float*, void*, void*, float*,
                 float*, float*, int, int, int, float, uint64_t, uint64_t, const uint64_t*, int, int, hipStream_t);
void pra_colsum16(const float*, void*, int, int, int, int, hipStream_t);
int pra_flash_fwd(const void*, const void*, const void*, void*, float*, int, int, int, int, int, const int64_t*, float,
                  int, int, hipStream_t);
int pra_flash_fwd_ext(const void*, const void*, const void*, void*, float*, int, int, int, int, int, const int64_t*,
                      float, int, int, const int*, const int*, const void*, int64_t, int64_t, int64_t, int, float,
                      uint64_t, uint64_t, uint32_t*, const uint64_t*, hipStream_t);
int pra_flash_bwd_ext(const void*, const void*, const void*, const void*, const float*, const float*, void*, void*,
                      void*, void*, int, int, int, int, int, const int64_t*, float, int, int, const int*, const int*,
                      const void*, int64_t, int64_t, int64_t, int, float, uint64_t, uint64_t, uint32_t*, const uint64_t*,
                      float*, hipStream_t);
int pra_flash_bwd(const void*, const void*, const void*, const void*, const void*, const float*, float*, void*, void*,
                  void*, void*, int, int, int, int, int, const int64_t*, float, int, int, float*, hipStream_t);
int pra_embedding_fwd(const int64_t*, const void*, void*, int64_t, int, int64_t, int64_t, int, hipStream_t);
int pra_embedding_bwd(const int64_t*, const int64_t*, const void*, void*, int64_t, int, int64_t, int64_t, int, int,
                      int, float*, hipStream_t);
void pra_bias_gelu_bwd_db(const void*, const void*, const void*, void*, float*, int, int, int, int, int,
                          hipStream_t);
void pra_colsum_rows(const void*, float*, int, int, int, int, hipStream_t);
int pra_colsum_multi(const float* const*, void* const*, const int*, int, int, int, int, hipStream_t);
int pra_bn_nrb(int, int);
int pra_max_pool_fwd(const void*, void*, uint8_t*, int, int, int, int, int, int, int, int, int, int, int, int, int,
                     hipStream_t);
int pra_max_pool_bwd(const void*, const uint8_t*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                     int, hipStream_t);
int pra_wflip_t(const void*, void*, int, int, int, int, int, hipStream_t);
int pra_gemm_bias_act(const void*, const void*, const void*, void*, void*, int, int, int, int, int, int, int, int,
                      hipStream_t);
int pra_gemm_lds(int, const void*, const void*, const void*, void*, void*, float*, int, int, int, int, int, int, int,
                 int, int, int, int, float*, hipStream_t);
int pra_gemm_lds_splits(int, int, int);
int pra_gemm_tn_grouped2(const void*, const void*, void*, int, int, int, int, const void*, const void*, void*, int, int,
                         int, int, int, int, int, hipStream_t);
void pra_gemm_set_w4(int);
void pra_gemm_set_pts(int);
int pra_gemm_get_pts();
void pra_spin_hog(int, long long, float*, hipStream_t);
int pra_gemm_probe(int, int, const void*, const void*, void*, int, int, int, int, int, int, unsigned long long*,
                   hipStream_t);
int pra_gemm_get_w4();
int pra_conv_lds(const void*, const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int,
                 int, float*, float*, const float*, int, hipStream_t, const void*, const uint8_t*, int);
int pra_conv_lds_stat_rows(int, int);
int pra_conv_dgrad_phase(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, float*,
                         const float*, const void*, const uint8_t*, hipStream_t);
int pra_conv_lds_splits(int, int, int);
int pra_conv_wgrad_rows(int);
int pra_conv_wgrad_lds(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, float*,
                       int, hipStream_t);
int pra_space_to_depth2(const void*, void*, int, int, int, int, int, int, int, hipStream_t);
int pra_colsum_partials(const float*, void*, int, int, int, hipStream_t);
void pra_bn_fwd_train(const void*, const void*, const void*, const void*, float*, float*, void*, uint8_t*, float*,
                      float*, float*, float*, int, int, int, float, float, int, int, int, hipStream_t);
void pra_bn_fwd_parts(const void*, const void*, const void*, const void*, float*, float*, void*, uint8_t*, float*,
                      float*, const float*, const float*, float*, int, int, int, float, float, int, int, int,
                      hipStream_t);
void pra_bn_fwd_infer(const void*, const void*, const void*, const void*, const float*, const float*, void*, float*,
                      int, int, float, int, int, int, hipStream_t);
void pra_bn_bwd(const void*, const void*, const uint8_t*, const void*, const void*, const float*, const float*, void*,
                void*, void*, void*, float*, float*, int, int, int, int, int, int, int, hipStream_t);
void pra_bn_premerge(const float*, float*, int, int, hipStream_t);
int pra_gap_bwd(const void*, void*, int, int, int, int, hipStream_t);
void pra_bn_bwd_parts(const void*, const void*, const void*, const float*, const float*, void*, void*, void*,
                      const float*, float*, int, int, int, int, int, int, hipStream_t);
}

#define V(x) reinterpret_cast<void*>(x)
#define CV(x) reinterpret_cast<const void*>(x)
#define F(x) reinterpret_cast<float*>(x)
#define CF(x) reinterpret_cast<const float*>(x)
#define I64(x) reinterpret_cast<const int64_t*>(x)
#define S(x) reinterpret_cast<hipStream_t>(x)

static void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

PYBIND11_MODULE(_pra_hip, m) {
  m.doc() = "paddle_ray_amd gfx950 HIP kernels";
  m.def("gemm_bias_act", [](P a, P b, P bias, P c, P z, int M, int N, int K, int lda, int ldb, int ldc, int dt, int act,
                            P s) {
    if (pra_gemm_bias_act(CV(a), CV(b), CV(bias), V(c), V(z), M, N, K, lda, ldb, ldc, dt, act, S(s)) != 0)
      throw std::invalid_argument("gemm_bias_act: unsupported shape/stride/dtype");
    check_launch("gemm_bias_act");
  });
  m.def("conv_lds", [](P x, P w, P bias, P y, int n, int h, int wd, int c, int cout, int kh, int kw, int st,
                       int pad, int relu, int dt, int splits, P ws, P part, P kshift, int pp, P s, P bnx, P bnmask,
                       int beta) {
    if (pra_conv_lds(CV(x), CV(w), CV(bias), V(y), n, h, wd, c, cout, kh, kw, st, pad, relu, dt, splits,
                     reinterpret_cast<float*>(ws), reinterpret_cast<float*>(part),
                     reinterpret_cast<const float*>(kshift), pp, S(s), CV(bnx),
                     reinterpret_cast<const uint8_t*>(bnmask), beta) != 0)
      throw std::invalid_argument("conv_lds: unsupported shape/dtype");
    check_launch("conv_lds");
  });
  m.def("conv_dgrad_phase", [](P dy, P wp, P dxp, int n, int ho, int wo, int co, int ci, int khp, int kwp, int os,
                               int dt, P part, P kshift, P bnx, P bnmask, P s) {
    if (pra_conv_dgrad_phase(CV(dy), CV(wp), V(dxp), n, ho, wo, co, ci, khp, kwp, os, dt, reinterpret_cast<float*>(part),
                             reinterpret_cast<const float*>(kshift), CV(bnx), reinterpret_cast<const uint8_t*>(bnmask),
                             S(s)) != 0)
      throw std::invalid_argument("conv_dgrad_phase: unsupported shape/dtype");
    check_launch("conv_dgrad_phase");
  });
  m.def("conv_wgrad_lds", [](P dy, P x, P dw, int n, int h, int wd, int c, int cout, int kh, int kw, int st, int pad,
                             int dt, int splits, P ws, int pp, P s) {
    if (pra_conv_wgrad_lds(CV(dy), CV(x), V(dw), n, h, wd, c, cout, kh, kw, st, pad, dt, splits,
                           reinterpret_cast<float*>(ws), pp, S(s)) != 0)
      throw std::invalid_argument("conv_wgrad_lds: unsupported shape/dtype");
    check_launch("conv_wgrad_lds");
  });
  m.def("space_to_depth2", [](P x, P y, int n, int h, int w, int c, int pad, int co, int dt, P s) {
    if (pra_space_to_depth2(CV(x), V(y), n, h, w, c, pad, co, dt, S(s)) != 0)
      throw std::invalid_argument("space_to_depth2: unsupported geometry");
    check_launch("space_to_depth2");
  });
  m.def("conv_lds_splits", [](int m, int n, int k) { return pra_conv_lds_splits(m, n, k); });
  m.def("conv_wgrad_rows", [](int cout) { return pra_conv_wgrad_rows(cout); });
  m.def("conv_lds_stat_rows", [](int m, int n) { return pra_conv_lds_stat_rows(m, n); });
  m.def("gemm_lds_splits", [](int M, int N, int K) { return pra_gemm_lds_splits(M, N, K); });
  m.def("gemm_set_w4", [](int mask) { pra_gemm_set_w4(mask); });
  m.def("gemm_set_pts", [](int mask) { pra_gemm_set_pts(mask); });
  m.def("gemm_get_pts", []() { return pra_gemm_get_pts(); });
  m.def("spin_hog", [](int nwg, long long cycles, P sink, P stream) { pra_spin_hog(nwg, cycles, (float*)sink, (hipStream_t)stream); });
  m.def("gemm_probe", [](int cfg, int layout, P a, P b, P c, int M, int N, int K, int lda, int ldb, int ldc, P st,
                         P stream) {
    return pra_gemm_probe(cfg, layout, CV(a), CV(b), V(c), M, N, K, lda, ldb, ldc,
                          reinterpret_cast<unsigned long long*>(st), S(stream));
  });
  m.def("gemm_get_w4", []() { return pra_gemm_get_w4(); });
  m.def("gemm_lds", [](int layout, P a, P b, P bias, P c, P z, P colsum, int M, int N, int K, int lda, int ldb,
                       int ldc, int ldz, int dt, int epi, int beta, int splits, P ws, P s) {
    if (pra_gemm_lds(layout, CV(a), CV(b), CV(bias), V(c), V(z), F(colsum), M, N, K, lda, ldb, ldc, ldz, dt, epi, beta,
                     splits, F(ws), S(s)) != 0)
      throw std::invalid_argument("gemm_lds: unsupported shape/stride/dtype");
    check_launch("gemm_lds");
  });
  m.def("gemm_tn_grouped2", [](P a1, P b1, P c1, int n1, int lda1, int ldb1, int ldc1, P a2, P b2, P c2, int n2,
                               int lda2, int ldb2, int ldc2, int M, int K, int beta, P s) {
    if (pra_gemm_tn_grouped2(CV(a1), CV(b1), V(c1), n1, lda1, ldb1, ldc1, CV(a2), CV(b2), V(c2), n2, lda2, ldb2, ldc2,
                             M, K, beta, S(s)) != 0)
      throw std::invalid_argument("gemm_tn_grouped2: unsupported shape");
    check_launch("gemm_tn_grouped2");
  });
  m.def("colsum_partials", [](P part, P out, int P_, int N, int dt, P s) {
    if (pra_colsum_partials(CF(part), V(out), P_, N, dt, S(s)) != 0)
      throw std::invalid_argument("colsum_partials: unsupported dtype");
    check_launch("colsum_partials");
  });
  m.def("layernorm_fwd", [](P x, P w, P b, P y, P mean, P rstd, int rows, int cols, float eps, int dtx, int dtw, P s) {
    pra_layernorm_fwd(CV(x), CV(w), CV(b), V(y), F(mean), F(rstd), rows, cols, eps, dtx, dtw, S(s));
    check_launch("layernorm_fwd");
  });
  m.def("layernorm_bwd", [](P dy, P x, P w, P mean, P rstd, P dx, P pw, P pb, int rows, int cols, int nblk, int dtx,
                            int dtw, P s) {
    pra_layernorm_bwd(CV(dy), CV(x), CV(w), CF(mean), CF(rstd), V(dx), F(pw), F(pb), rows, cols, nblk, dtx, dtw, S(s));
    check_launch("layernorm_bwd");
  });
  m.def("rmsnorm_fwd", [](P x, P w, P y, P rstd, int rows, int cols, float eps, int dtx, int dtw, P s) {
    pra_rmsnorm_fwd(CV(x), CV(w), V(y), F(rstd), rows, cols, eps, dtx, dtw, S(s));
    check_launch("rmsnorm_fwd");
  });
  m.def("rmsnorm_bwd", [](P dy, P x, P w, P rstd, P dx, P pw, int rows, int cols, int nblk, int dtx, int dtw, P s) {
    pra_rmsnorm_bwd(CV(dy), CV(x), CV(w), CF(rstd), V(dx), F(pw), rows, cols, nblk, dtx, dtw, S(s));
    check_launch("rmsnorm_bwd");
  });
  m.def("colsum", [](P part, P out, int nblk, int cols, int dt, P s) {
    pra_colsum(CF(part), V(out), nblk, cols, dt, S(s));
    check_launch("colsum");
  });
  m.def("softmax_fwd", [](P x, P y, int rows, int cols, int dt, P s) {
    pra_softmax_fwd(CV(x), V(y), rows, cols, dt, S(s));
    check_launch("softmax_fwd");
  });
  m.def("softmax_bwd", [](P y, P dy, P dx, int rows, int cols, int dt, P s) {
    pra_softmax_bwd(CV(y), CV(dy), V(dx), rows, cols, dt, S(s));
    check_launch("softmax_bwd");
  });
  m.def("softmax_ce_fwd", [](P logits, P labels, P loss, P lse, int rows, int V_, int ign, int dt, P s) {
    pra_softmax_ce_fwd(CV(logits), I64(labels), F(loss), F(lse), rows, V_, ign, dt, S(s));
    check_launch("softmax_ce_fwd");
  });
  m.def("softmax_ce_bwd", [](P logits, P labels, P lse, P dloss, P dl, int rows, int V_, int ign, int dt, P s) {
    pra_softmax_ce_bwd(CV(logits), I64(labels), CF(lse), CF(dloss), V(dl), rows, V_, ign, dt, S(s));
    check_launch("softmax_ce_bwd");
  });
  m.def("vp_ce_part_fwd", [](P logits, P labels, P stats, int rows, int V_, int64_t start, int dt, P s) {
    pra_vp_ce_part_fwd(CV(logits), I64(labels), F(stats), rows, V_, start, dt, S(s));
    check_launch("vp_ce_part_fwd");
  });
  m.def("vp_ce_final", [](P stats, P labels, P loss, P lse, int rows, int world, int64_t vtot, int ign, P s) {
    pra_vp_ce_final(CF(stats), I64(labels), F(loss), F(lse), rows, world, vtot, ign, S(s));
    check_launch("vp_ce_final");
  });
  m.def("vp_ce_bwd", [](P logits, P labels, P lse, P dloss, P dl, int rows, int V_, int64_t start, int64_t vtot,
                        int ign, int dt, P s) {
    pra_vp_ce_bwd(CV(logits), I64(labels), CF(lse), CF(dloss), V(dl), rows, V_, start, vtot, ign, dt, S(s));
    check_launch("vp_ce_bwd");
  });
  m.def("build_info", []() { return std::string(pra_build_info()); });
  // id of the stream capture in progress on s (0 when s is not capturing): the graph-safe dropout
  // RNG advances its device step counter once per capture (ops/fused.py _graph_seq)
  m.def("capture_id", [](P s) -> unsigned long long {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    if (hipStreamGetCaptureInfo(S(s), &st, &id) != hipSuccess || st != hipStreamCaptureStatusActive) return 0ull;
    return id;
  });
  m.def("mmha_splits", [](int B, int H, int t) { return pra_mmha_splits(B, H, t); });
  m.def("mmha_decode", [](P qkv, P cache, P mask, P ws, P out, int B, int H, int L, int D, int t, P t_dev,
                          int splits, int mask_len, float scale, int dt, P s) {
    if (pra_mmha_decode(CV(qkv), V(cache), CF(mask), F(ws), V(out), B, H, L, D, t,
                        reinterpret_cast<const int*>(t_dev), splits, mask_len, scale, dt, S(s)) != 0)
      throw std::invalid_argument("mmha_decode: unsupported head_dim/dtype or time_step out of range");
    check_launch("mmha_decode");
  });
  m.def("bias_gelu_fwd", [](P x, P b, P y, int64_t rows, int cols, int dt, int approx, P s) {
    pra_bias_gelu_fwd(CV(x), CV(b), V(y), rows, cols, dt, approx, S(s));
    check_launch("bias_gelu_fwd");
  });
  m.def("bias_gelu_bwd", [](P dy, P x, P b, P dx, int64_t rows, int cols, int dt, int approx, P s) {
    pra_bias_gelu_bwd(CV(dy), CV(x), CV(b), V(dx), rows, cols, dt, approx, S(s));
    check_launch("bias_gelu_bwd");
  });
  m.def("zero_mt", [](P chunks, int n, P s) {
    pra_zero_mt(I64(chunks), n, S(s));
    check_launch("zero_mt");
  });
  m.def("adamw_mt", [](P tab, P ftab, P chunks, int nch, float lr, float b1, float b2, float eps, float bc1, float bc2,
                       float gs, P s, P gsp) {
    pra_adamw_mt(I64(tab), CF(ftab), I64(chunks), nch, lr, b1, b2, eps, bc1, bc2, gs, CF(gsp), S(s));
    check_launch("adamw_mt");
  });
  m.def("momentum_mt", [](P tab, P ftab, P chunks, int nch, float lr, float mu, int nesterov, float gs, P s,
                          P gsp) {
    pra_momentum_mt(I64(tab), CF(ftab), I64(chunks), nch, lr, mu, nesterov, gs, CF(gsp), S(s));
    check_launch("momentum_mt");
  });
  m.def("lamb_shard_stage1", [](P pieces, int np_, P g, int gdt, P w, P m_, P v, P r, P wd, P norms, int nparams,
                                float b1, float b2, float eps, float bc1, float bc2, float gs, P gsp, P s) {
    pra_lamb_shard_stage1(I64(pieces), np_, CV(g), gdt, CF(w), F(m_), F(v), F(r), CF(wd), F(norms), nparams, b1, b2,
                          eps, bc1, bc2, gs, CF(gsp), S(s));
    check_launch("lamb_shard_stage1");
  });
  m.def("lamb_shard_stage2", [](P pieces, int np_, P w, P r, P norms, int nparams, float lr, P pout, int pdt, P s) {
    pra_lamb_shard_stage2(I64(pieces), np_, F(w), CF(r), CF(norms), nparams, lr, reinterpret_cast<void*>(pout), pdt,
                          S(s));
    check_launch("lamb_shard_stage2");
  });
  m.def("sumsq_accum", [](P x, P out, int64_t n, int dt, P s) {
    pra_sumsq_accum(CV(x), F(out), n, dt, S(s));
    check_launch("sumsq_accum");
  });
  m.def("adl_supported", [](int cols) { return pra_adl_supported(cols); });
  m.def("adl_fwd", [](P x, P h, P hb, P w, P b, P r, P y, P mean, P rstd, int rows, int cols, float eps, float p,
                      uint64_t seed, uint64_t off, P dseq, int dt, int dtw, P s) {
    pra_adl_fwd(CV(x), CV(h), CV(hb), CV(w), CV(b), V(r), V(y), F(mean), F(rstd), rows, cols, eps, p, seed, off,
                reinterpret_cast<const uint64_t*>(dseq), dt, dtw, S(s));
    check_launch("adl_fwd");
  });
  m.def("adl_bwd", [](P dy, P dro, P r, P w, P mean, P rstd, P dri, P dh, P pw, P pb, P pbias, int rows, int cols,
                      int nblk, float p, uint64_t seed, uint64_t off, P dseq, int dt, int dtw, P s) {
    pra_adl_bwd(CV(dy), CV(dro), CV(r), CV(w), CF(mean), CF(rstd), V(dri), V(dh), F(pw), F(pb), F(pbias), rows, cols,
                nblk, p, seed, off, reinterpret_cast<const uint64_t*>(dseq), dt, dtw, S(s));
    check_launch("adl_bwd");
  });
  m.def("colsum16", [](P part, P out, int nblk, int cols, int dt, P s) {
    pra_colsum16(CF(part), V(out), nblk, cols, dt, 0, S(s));
    check_launch("colsum16");
  });
  m.def("colsum16_acc", [](P part, P out, int nblk, int cols, int dt, P s) {
    pra_colsum16(CF(part), V(out), nblk, cols, dt, 1, S(s));
    check_launch("colsum16_acc");
  });
  m.def("flash_bwd_pre", [](P o, P dO, P delta, int B, int H, int Sq, int D, int dt, P s) {
    pra_flash_bwd_pre(CV(o), CV(dO), F(delta), B, H, Sq, D, dt, S(s));
    check_launch("flash_bwd_pre");
  });
  m.def("flash_fwd", [](P q, P k, P v, P o, P lse, int B, int H, int Sq, int Sk, int D, int64_t qsb, int64_t qss,
                        int64_t qsh, int64_t ksb, int64_t kss, int64_t ksh, int64_t vsb, int64_t vss, int64_t vsh,
                        float scale, int causal, int dt, P s) {
    int64_t st[9] = {qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh};
    if (pra_flash_fwd(CV(q), CV(k), CV(v), V(o), F(lse), B, H, Sq, Sk, D, st, scale, causal, dt, S(s)) != 0)
      throw std::invalid_argument("flash_fwd: unsupported head_dim/dtype");
    check_launch("flash_fwd");
  });
  m.def("flash_fwd_ext", [](P q, P k, P v, P o, P lse, int B, int H, int Sq, int Sk, int D, std::vector<int64_t> st,
                            float scale, int causal, int dt, P cu_q, P cu_k, P mask, int64_t msb, int64_t msh,
                            int64_t msq, int mask_f32, float p_drop, uint64_t seed, uint64_t offset, P dbits, P dseq,
                            P s) {
    if (st.size() != 9) throw std::invalid_argument("flash_fwd_ext: need 9 strides");
    if (pra_flash_fwd_ext(CV(q), CV(k), CV(v), V(o), F(lse), B, H, Sq, Sk, D, st.data(), scale, causal, dt,
                          reinterpret_cast<const int*>(cu_q), reinterpret_cast<const int*>(cu_k), CV(mask), msb, msh,
                          msq, mask_f32, p_drop, seed, offset, reinterpret_cast<uint32_t*>(dbits),
                          reinterpret_cast<const uint64_t*>(dseq), S(s)) != 0)
      throw std::invalid_argument("flash_fwd_ext: unsupported arguments");
    check_launch("flash_fwd_ext");
  });
  m.def("flash_bwd_ext", [](P q, P k, P v, P dO, P lse, P delta, P dq, P dk, P dv, P dsT, int B, int H, int Sq, int Sk,
                            int D, std::vector<int64_t> st, float scale, int causal, int dt, P cu_q, P cu_k, P mask,
                            int64_t msb, int64_t msh, int64_t msq, int mask_f32, float p_drop, uint64_t seed,
                            uint64_t offset, P dbits, P dseq, P s, P bsum) {
    if (st.size() != 18) throw std::invalid_argument("flash_bwd_ext: need 18 strides");
    if (pra_flash_bwd_ext(CV(q), CV(k), CV(v), CV(dO), CF(lse), CF(delta), V(dq), V(dk), V(dv), V(dsT), B, H, Sq, Sk,
                          D, st.data(), scale, causal, dt, reinterpret_cast<const int*>(cu_q),
                          reinterpret_cast<const int*>(cu_k), CV(mask), msb, msh, msq, mask_f32, p_drop, seed,
                          offset, reinterpret_cast<uint32_t*>(dbits), reinterpret_cast<const uint64_t*>(dseq),
                          F(bsum), S(s)) != 0)
      throw std::invalid_argument("flash_bwd_ext: unsupported arguments");
    check_launch("flash_bwd_ext");
  });
  m.def("flash_bwd", [](P q, P k, P v, P dO, P o, P lse, P delta, P dq, P dk, P dv, P dsT, int B, int H, int Sq,
                        int Sk, int D, std::vector<int64_t> st, float scale, int causal, int dt, P s, P bsum) {
    if (st.size() != 18) throw std::invalid_argument("flash_bwd: need 18 strides");
    if (pra_flash_bwd(CV(q), CV(k), CV(v), CV(dO), CV(o), CF(lse), F(delta), V(dq), V(dk), V(dv), V(dsT), B, H, Sq, Sk, D, st.data(),
                      scale, causal, dt, F(bsum), S(s)) != 0)
      throw std::invalid_argument("flash_bwd: unsupported head_dim/dtype");
    check_launch("flash_bwd");
  });
  m.def("bn_nrb", [](int M, int C) { return pra_bn_nrb(M, C); });
  m.def("bn_fwd_train", [](P x, P z, P w, P b, P rm, P rv, P y, P mask, P mean, P invstd, P part, P coef, int M,
                           int C, int nrb, float eps, float mom, int relu, int dt, int dtw, P s) {
    pra_bn_fwd_train(CV(x), CV(z), CV(w), CV(b), F(rm), F(rv), V(y), reinterpret_cast<uint8_t*>(mask), F(mean),
                     F(invstd), F(part), F(coef), M, C, nrb, eps, mom, relu, dt, dtw, S(s));
    check_launch("bn_fwd_train");
  });
  m.def("bn_fwd_parts", [](P x, P z, P w, P b, P rm, P rv, P y, P mask, P mean, P invstd, P part, P kshift, P coef,
                           int M, int C, int nrb, float eps, float mom, int relu, int dt, int dtw, P s) {
    pra_bn_fwd_parts(CV(x), CV(z), CV(w), CV(b), F(rm), F(rv), V(y), reinterpret_cast<uint8_t*>(mask), F(mean),
                     F(invstd), reinterpret_cast<const float*>(part), reinterpret_cast<const float*>(kshift), F(coef),
                     M, C, nrb, eps, mom, relu, dt, dtw, S(s));
    check_launch("bn_fwd_parts");
  });
  m.def("bn_fwd_infer", [](P x, P z, P w, P b, P rm, P rv, P y, P coef, int M, int C, float eps, int relu, int dt,
                           int dtw, P s) {
    pra_bn_fwd_infer(CV(x), CV(z), CV(w), CV(b), CF(rm), CF(rv), V(y), F(coef), M, C, eps, relu, dt, dtw, S(s));
    check_launch("bn_fwd_infer");
  });
  m.def("bn_bwd", [](P dy, P y, P mask, P x, P w, P mean, P invstd, P dx, P dz, P dw, P db, P part, P coef, int M,
                     int C, int nrb, int relu, int dt, int dtw, int acc, P s) {
    pra_bn_bwd(CV(dy), CV(y), reinterpret_cast<const uint8_t*>(mask), CV(x), CV(w), CF(mean), CF(invstd), V(dx), V(dz),
               V(dw), V(db), F(part), F(coef), M, C, nrb, relu, dt, dtw, acc, S(s));
    check_launch("bn_bwd");
  });
  m.def("gap_bwd", [](P dy, P dx, int n, int hw, int c, int dt, P s) {
    if (pra_gap_bwd(CV(dy), V(dx), n, hw, c, dt, S(s)) != 0) throw std::invalid_argument("gap_bwd: unsupported shape");
    check_launch("gap_bwd");
  });
  m.def("bn_premerge", [](P part, P out, int nrb, int C, P s) {
    pra_bn_premerge(reinterpret_cast<const float*>(part), F(out), nrb, C, S(s));
    check_launch("bn_premerge");
  });
  m.def("bn_bwd_parts", [](P g, P x, P w, P mean, P invstd, P dx, P dw, P db, P part, P coef, int M, int C, int nrb,
                           int dt, int dtw, int acc, P s) {
    pra_bn_bwd_parts(CV(g), CV(x), CV(w), CF(mean), CF(invstd), V(dx), V(dw), V(db),
                     reinterpret_cast<const float*>(part), F(coef), M, C, nrb, dt, dtw, acc, S(s));
    check_launch("bn_bwd_parts");
  });
  m.def("max_pool_fwd", [](P x, P y, P idx, int n, int h, int w, int c, int ho, int wo, int kh, int kw, int sh,
                           int sw, int ph, int pw, int dt, P s) {
    if (pra_max_pool_fwd(CV(x), V(y), reinterpret_cast<uint8_t*>(idx), n, h, w, c, ho, wo, kh, kw, sh, sw, ph, pw, dt,
                         S(s)) != 0)
      throw std::invalid_argument("max_pool_fwd: unsupported geometry");
    check_launch("max_pool_fwd");
  });
  m.def("max_pool_bwd", [](P dy, P idx, P dx, int n, int h, int w, int c, int ho, int wo, int kh, int kw, int sh,
                           int sw, int ph, int pw, int dt, P s) {
    if (pra_max_pool_bwd(CV(dy), reinterpret_cast<const uint8_t*>(idx), V(dx), n, h, w, c, ho, wo, kh, kw, sh, sw, ph,
                         pw, dt, S(s)) != 0)
      throw std::invalid_argument("max_pool_bwd: unsupported geometry");
    check_launch("max_pool_bwd");
  });
  m.def("wflip_t", [](P src, P dst, int o, int c, int kh, int kw, int dt, P s) {
    if (pra_wflip_t(CV(src), V(dst), o, c, kh, kw, dt, S(s)) != 0)
      throw std::invalid_argument("wflip_t: unsupported shape");
    check_launch("wflip_t");
  });
  m.def("embedding_fwd", [](P ids, P w, P out, int64_t n, int D, int64_t V, int64_t pad, int dt, P s) {
    if (pra_embedding_fwd(I64(ids), CV(w), V(out), n, D, V, pad, dt, S(s)) != 0)
      throw std::invalid_argument("embedding_fwd: unsupported D/dtype");
    check_launch("embedding_fwd");
  });
  m.def("embedding_bwd", [](P sids, P perm, P dy, P dw, int64_t n, int D, int64_t V, int64_t pad, int dtg, int dtw,
                            int acc, P ws, P s) {
    if (pra_embedding_bwd(I64(sids), I64(perm), CV(dy), V(dw), n, D, V, pad, dtg, dtw, acc, F(ws), S(s)) != 0)
      throw std::invalid_argument("embedding_bwd: unsupported D/dtype");
    check_launch("embedding_bwd");
  });
  m.def("bias_gelu_bwd_db", [](P dy, P x, P b, P dx, P part, int rows, int cols, int nrb, int dt, int approx,
                               P s) {
    pra_bias_gelu_bwd_db(CV(dy), CV(x), CV(b), V(dx), F(part), rows, cols, nrb, dt, approx, S(s));
    check_launch("bias_gelu_bwd_db");
  });
  m.def("colsum_multi", [](std::vector<P> parts, std::vector<P> outs, std::vector<int> accs, int nblk, int cols,
                           int dt, P s) {
    const int n = (int)parts.size();
    if (n != (int)outs.size() || n != (int)accs.size() || n < 1 || n > 3)
      throw std::invalid_argument("colsum_multi: 1-3 jobs with matching lists");
    const float* pp[3];
    void* po[3];
    for (int j = 0; j < n; ++j) { pp[j] = CF(parts[j]); po[j] = V(outs[j]); }
    if (pra_colsum_multi(pp, po, accs.data(), n, nblk, cols, dt, S(s)) != 0)
      throw std::invalid_argument("colsum_multi: unsupported shape/alignment");
    check_launch("colsum_multi");
  });
  m.def("colsum_rows", [](P x, P part, int rows, int cols, int nrb, int dt, P s) {
    if (cols % 8) throw std::invalid_argument("colsum_rows: cols % 8 != 0");
    pra_colsum_rows(CV(x), F(part), rows, cols, nrb, dt, S(s));
    check_launch("colsum_rows");
  });
}
