// LDS-DMA pipelined MFMA GEMM for gfx950 (CDNA4) — the framework's training GEMM.
//
//   C[M,N] (=|+=) epi( A[M,K] · B[K,N] )     bf16/f16 operands, fp32 accumulation
//
// Operand layouts (template flags), covering the three GEMMs of a Linear layer with Paddle's
// [in, out] weight (reference python/paddle/nn/functional/common.py `linear`; the fused
// epilogues follow paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue_kernel.cu semantics):
//   AK = true : A stored [M][K] (row pitch lda)  — "K-contiguous"
//   AK = false: A stored [K][M] (row pitch lda)  — "M-contiguous"
//   BK = true : B stored [N][K] (row pitch ldb)
//   BK = false: B stored [K][N] (row pitch ldb)
//   forward  y = x·W        : AK=1, BK=0     dgrad dx = dy·Wᵀ : AK=1, BK=1
//   wgrad   dW = xᵀ·dy      : AK=0, BK=0     (tied LM head: logits = h·Eᵀ is AK=1, BK=1)
//
// Structure (cdna_hip_programming.md §5: glds staging pipeline, counted vmcnt, raw barrier):
//   * 256x256 output tile per 512-thread workgroup (8 wave64 = 2(M) x 4(N), 128x64 per wave,
//     8x4 accumulators of v_mfma_f32_16x16x32_{bf16,f16}); 1 workgroup per CU.
//   * K is staged 64 deep per step (whole 128-B lines of every row) into 2 LDS slots (2 x 64 KB) by
//     global_load_lds_dwordx4 (LDS-DMA: no VGPR staging, no ds_write). The step-(k+2) DMA is
//     issued under step k's second k-half; fragments are register double-buffered per 32-deep
//     k-half so every LDS read runs under the previous half's MFMAs; one raw s_barrier per
//     K-step (no __syncthreads: its fence would drain the DMA).
//   * LDS images are lane-linear (what LDS-DMA writes); bank swizzles are applied by permuting
//     each lane's GLOBAL source chunk and reading with the same permutation:
//       K-contiguous operand -> image [row][32 k] (64-B rows), 16-B chunk ^= kc_swz(row),
//                               fragments by ds_read_b128 (conflict-free in its lane groups);
//       MN-contiguous operand -> image [k][256] (512-B rows), chunk ^= 2*((k&3)|((k>>1)&4)),
//                               fragments by 2 x ds_read_b64_tr_b16 (hardware transpose).
//   * MFMAs are issued as (B-frag, A-frag) so each lane's accumulator holds 4 consecutive
//     output COLUMNS of one row -> packed 8-byte epilogue stores.
//   * XCD-aware bijective tile remap + 8-row tile grouping for L2 reuse.
// Epilogue (in registers on the accumulators): + bias[N], activation (GELU tanh/erf, ReLU)
// with the pre-activation optionally stored to Z, or dGELU: C = acc * gelu'(Z) with per-tile
// column partial sums written to `colsum` (the bias gradient, reduced by pra_colsum_partials);
// `beta=1` accumulates into C (dW += xᵀ·dy straight into the flat gradient buffer).
#include "gemm_core.h"

extern "C" int pra_gemm_alt(int cfg, int layout, const void* A, const void* B, const void* bias, void* C, void* Z,
                            float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype, int epi,
                            int beta, int splits, float* ws, hipStream_t s);

extern "C" int pra_gemm_pts_w4(int layout, const void* A, const void* B, const void* bias, void* C, void* Z,
                               float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype,
                               int epi, int beta, hipStream_t s);
extern "C" int pra_gemm_pts_w4b(int layout, const void* A, const void* B, const void* bias, void* C, void* Z,
                                float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype,
                                int epi, int beta, hipStream_t s);
extern "C" int pra_gemm_pts_w8(int layout, const void* A, const void* B, const void* bias, void* C, void* Z,
                               float* colsum, int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype,
                               int epi, int beta, hipStream_t s);

namespace pra {
namespace {

// Persistent TS kernel (gemm_pts.h) per layout, bit = 1 << layout: one workgroup per CU walks
// its tiles with the next tile's operand DMA overlapping the epilogue. dy·Wᵀ runs the 4-wave
// configuration (bit 4 of the mask switches it to 8 waves), x·W and xᵀ·dy the 8-wave one.
// PRA_GEMM_PTS at first use (default 0 until measured; 7: every layout), pra_gemm_set_pts afterwards.
int g_pts_mask = -1;
// per call: epi bit 8 (kPersistBit) asks for the persistent kernel regardless of the mask (the
// framework's shape policy picks it for short-K dy·Wᵀ, where it measured ahead of hipBLASLt)
constexpr int kPersistBit = 256;
thread_local bool g_force_pts = false;
int pts_mask() {
  if (g_pts_mask < 0) {
    const char* e = getenv("PRA_GEMM_PTS");
    g_pts_mask = e ? atoi(e) : 0;
  }
  return g_pts_mask;
}

// Which layouts run an alternative configuration of gemm_w4.hip, 4 mask bits per config
// (bit = 1 << (4 * cfg + layout)): cfg 0 = W4 (4 waves x 128x128), 1 = W8I (8 waves, one filler
// per MFMA), 2 = W4B (W4 with MUBUF operand DMA), 3 = W8B (W8 with MUBUF operand DMA),
// 4 = W4P / 5 = W8P (two barriers per K-step, refill DMA issued in half 0).
// 6 = W4T / 7 = W8T (the TS schedule: reads of a K-step early, refill spread one piece per 5 / 4
// MFMAs, counted vmcnt late; gemm_core.h kstep_t).
// Default (profiles/r4g/ts.log, 15 GPT shapes): W8T for x·W and xᵀ·dy, W4T for dy·Wᵀ -- 1.8-2 %
// under the W8 baseline overall, best on 13 of 15 shapes.
// PRA_GEMM_W4 at first use (0 = the W8 baseline), pra_gemm_set_w4 afterwards (A/B timing in one process).
constexpr int kDefaultAltMask = (1 << (4 * 7 + 0)) | (1 << (4 * 6 + 1)) | (1 << (4 * 7 + 2));
int g_w4_mask = -1;
int w4_mask() {
  if (g_w4_mask < 0) {
    const char* e = getenv("PRA_GEMM_W4");
    g_w4_mask = e ? atoi(e) : kDefaultAltMask;
  }
  return g_w4_mask;
}

// 128 x 256 tiles (8 waves of 64 x 64, 128-wide M-contiguous dy image) for weight gradients with
// at most 128 output rows (narrow convolutions, Cout <= 128), where the 256-row tile idles half or
// more of its MFMA rows. PRA_GEMM_NARROW=0 keeps the TN GEMMs on the 256-row tile (A/B).
using WG128 = WCfg<2, 4, 128, 256>;
bool narrow_tn() {
  static const bool on = !getenv("PRA_GEMM_NARROW") || atoi(getenv("PRA_GEMM_NARROW")) != 0;
  return on;
}

template <typename T, bool AK, bool BK, int E>
void launch_e(const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum, int M, int N, int K,
              int lda, int ldb, int ldc, int ldz, int beta, int splits, float* ws, hipStream_t s) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  auto pa = static_cast<const uint16_t*>(A);
  auto pb = static_cast<const uint16_t*>(B);
  auto pbias = static_cast<const uint16_t*>(bias);
  auto pc = static_cast<uint16_t*>(C);
  auto pz = static_cast<uint16_t*>(Z);
  // alternative configurations (gemm_w4.hip) per layout mask: W4's round-2 measurement (12-45 %
  // slower) was taken with the accumulators spilled to scratch by the compiler; round 3
  // (profiles/r3_gemm): W4 / W8I within +-3 % of W8, hipBLASLt still ahead on dy·Wᵀ.
  static const int ablate = getenv("PRA_GEMM_ABLATE") ? 0 : 1;  // 0: no DMA after the prologue (timing only)
  constexpr int layout = AK ? (BK ? 1 : 0) : 2;
  int alt = -1;
  if (std::is_same<T, bf16>::value && E != kRelu)
    for (int c = 0; c < 8 && alt < 0; ++c)
      if (w4_mask() >> (4 * c + layout) & 1) alt = c;
  // TN GEMMs with <= 128 rows (one tile row either way, so split-K factors and workspaces match)
  const bool narrow = !AK && !BK && E == kNone && M <= 128 && alt < 0 && narrow_tn();
  if (splits > 1) {
    if (alt >= 0)
      pra_gemm_alt(alt, layout, A, B, nullptr, nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, ldz, kBF16, 0, 0,
                   splits, ws, s);
    else if (narrow)
      gemm_lds_kernel<T, WG128, AK, BK, kNone, false, true><<<tiles * splits, WG128::NT, 0, s>>>(
          pa, pb, nullptr, nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, ldz, splits, ws);
    else
      gemm_lds_kernel<T, W8, AK, BK, kNone, false, true><<<tiles * splits, W8::NT, 0, s>>>(
          pa, pb, nullptr, nullptr, nullptr, nullptr, M, N, K, lda, ldb, ldc, ldz, splits, ws);
    const int64_t quads = (int64_t)M * N / 4;
    const int G = splitk_groups(quads, splits);
    const int blocks = (int)((quads * G + 255) / 256);
    if (beta) splitk_reduce_k<T, E, true><<<blocks, 256, 0, s>>>(ws, splits, pbias, pc, pz, M, N, ldc, ldz, G);
    else splitk_reduce_k<T, E, false><<<blocks, 256, 0, s>>>(ws, splits, pbias, pc, pz, M, N, ldc, ldz, G);
    return;
  }
  // (measured: front-loading the step's DMA into the first 2 / 4 segments of the half instead of
  // one per segment was 1-10 % slower on every GPT shape)
  // (measured: one static s_setprio 1 for waves 4-7 instead of the per-segment flips is neutral,
  // 11.65 vs 11.60 ms over the 15 GPT shapes, 131.2 vs 131.1-131.3 ms per GPT step)
#define PRA_GEMM_LAUNCH(CFG, BETA_)                                                                         \
  gemm_lds_kernel<T, CFG, AK, BK, E, BETA_, false><<<tiles, CFG::NT, 0, s>>>(pa, pb, pbias, pc, pz, colsum, M, N, K, \
                                                                           lda, ldb, ldc, ldz, ablate, nullptr)
  if (std::is_same<T, bf16>::value && E != kRelu && (g_force_pts || (pts_mask() >> layout & 1))) {
    // 4 waves (128x128 per wave, AGPR accumulators) for dy·Wᵀ unless mask bit 16, and for x·W
    // with mask bit 32 or a per-call persistent request (the fused GELU forward: 486 vs 517 us
    // per-tile at 16384 x 8192 x 2048, profiles/r5/gemm_fwd_probe.log); 8 waves otherwise
    const bool w4 = (layout == 1 && !(pts_mask() & 16)) || (layout == 0 && ((pts_mask() & 32) || g_force_pts));
    static const bool buf = getenv("PRA_PTS_BUF") && atoi(getenv("PRA_PTS_BUF")) == 1;
    if ((w4 ? (buf ? pra_gemm_pts_w4b : pra_gemm_pts_w4) : pra_gemm_pts_w8)(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, kBF16,
                                                 E, beta, s) == 0)
      return;
  }
  if (alt >= 0 && pra_gemm_alt(alt, layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, kBF16, E, beta, 1,
                               nullptr, s) == 0)
    return;
  if constexpr (!AK && !BK && E == kNone) {
    if (narrow) {
      if (beta) PRA_GEMM_LAUNCH(WG128, true); else PRA_GEMM_LAUNCH(WG128, false);
      return;
    }
  }
  if (beta) PRA_GEMM_LAUNCH(W8, true); else PRA_GEMM_LAUNCH(W8, false);
#undef PRA_GEMM_LAUNCH
}

template <typename T, bool AK, bool BK>
int launch_l(const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum, int M, int N, int K,
             int lda, int ldb, int ldc, int ldz, int epi, int beta, int splits, float* ws, hipStream_t s) {
  switch (epi) {
    case kNone: launch_e<T, AK, BK, kNone>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break;
    case kGeluErf: launch_e<T, AK, BK, kGeluErf>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break;
    case kGeluTanh: launch_e<T, AK, BK, kGeluTanh>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break;
    case kRelu: launch_e<T, AK, BK, kRelu>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break;
    case kDGeluErf: launch_e<T, AK, BK, kDGeluErf>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break;
    case kDGeluTanh: launch_e<T, AK, BK, kDGeluTanh>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break;
    // derivative-saving forward GELU (x·W only) and its multiply-by-Z dgrad (dy·Wᵀ only)
    case kGeluErfD:
      if constexpr (AK && !BK) { launch_e<T, AK, BK, kGeluErfD>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break; }
      return -1;
    case kGeluTanhD:
      if constexpr (AK && !BK) { launch_e<T, AK, BK, kGeluTanhD>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break; }
      return -1;
    case kMulZ:
      if constexpr (AK && BK) { launch_e<T, AK, BK, kMulZ>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, beta, splits, ws, s); break; }
      return -1;
    default: return -1;
  }
  return 0;
}

template <typename T>
int launch_t(int layout, const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum, int M, int N,
             int K, int lda, int ldb, int ldc, int ldz, int epi, int beta, int splits, float* ws, hipStream_t s) {
  switch (layout) {
    case 0: return launch_l<T, true, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, splits, ws, s);
    case 1: return launch_l<T, true, true>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, splits, ws, s);
    case 2: return launch_l<T, false, false>(A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, splits, ws, s);
    default: return -1;
  }
}

template <typename T, typename CF, int E>
void launch_conv_cfg(const void* xpad, const void* W, const void* bias, void* Y, int M, int N, int K,
                     const ConvGeom& cg, int splits, float* ws, float* part, const float* kshift, hipStream_t s,
                     const void* bnx = nullptr, const uint8_t* bnmask = nullptr, int beta = 0) {
  const int tiles_m = (M + CF::BM - 1) / CF::BM;
  const int tiles = tiles_m * ((N + CF::BN - 1) / CF::BN);
  auto px = static_cast<const uint16_t*>(xpad);
  auto pw = static_cast<const uint16_t*>(W);
  auto pb = static_cast<const uint16_t*>(bias);
  auto py = static_cast<uint16_t*>(Y);
  if constexpr (E != kBnG) {
    if (splits > 1) {  // few output tiles (late ResNet stages): split the K = KH*KW*C loop
      gemm_lds_kernel<T, CF, true, true, kNone, false, true, true><<<tiles * splits, CF::NT, 0, s>>>(
          px, pw, nullptr, nullptr, nullptr, nullptr, M, N, K, 0, K, N, N, splits, ws, cg);
      const int64_t quads = (int64_t)M * N / 4;
      const int G = splitk_groups(quads, splits);
      splitk_reduce_k<T, E, false><<<(int)((quads * G + 255) / 256), 256, 0, s>>>(ws, splits, pb, py, nullptr, M, N,
                                                                                 N, N, G);
      return;
    }
  }
  // part (optional): per-tile-row BatchNorm statistics of the output, [2][tiles_m][N] = sums of
  // (y - kshift) and (y - kshift)^2 over each tile's rows (kshift: the running mean).
  // kBnG: Y = dgrad masked by bnmask, part = sums of Y and Y * (bnx - kshift) (kshift: BN batch mean)
  if constexpr (E == kBnG) {
    if (beta) {  // the pending gradient in Y is added before the ReLU mask (a residual join's last term)
      gemm_lds_kernel<T, CF, true, true, E, true, false, true><<<tiles, CF::NT, 0, s>>>(
          px, pw, pb, py, const_cast<uint16_t*>(static_cast<const uint16_t*>(bnx)), part, M, N, K, 0, K, N, N, 1,
          nullptr, cg, part + (int64_t)tiles_m * N, kshift, bnmask);
      return;
    }
  }
  gemm_lds_kernel<T, CF, true, true, E, false, false, true><<<tiles, CF::NT, 0, s>>>(
      px, pw, pb, py, const_cast<uint16_t*>(static_cast<const uint16_t*>(bnx)), part, M, N, K, 0, K, N, N, 1, nullptr,
      cg, part ? part + (int64_t)tiles_m * N : nullptr, kshift, bnmask);
}

inline int conv_wgrad_rows(int Cout) { return Cout <= 128 ? WG128::BM : W8::BM; }

// dW [Cout][KH*KW*C] = dy[pix][Cout]ᵀ · im2col(x)[pix][KH*KW*C] (TN, gathered B), split-K over pixels
template <typename T, typename CF>
void launch_conv_wgrad_cfg(const void* dy, const void* x, void* dW, int Mpix, int Cout, int Nk, const ConvGeom& cg,
                           int splits, float* ws, hipStream_t s) {
  const int tiles = ((Cout + CF::BM - 1) / CF::BM) * ((Nk + CF::BN - 1) / CF::BN);
  auto pdy = static_cast<const uint16_t*>(dy);
  auto px = static_cast<const uint16_t*>(x);
  auto pw = static_cast<uint16_t*>(dW);
  if (splits > 1) {
    gemm_lds_kernel<T, CF, false, false, kNone, false, true, false, 0, true><<<tiles * splits, CF::NT, 0, s>>>(
        pdy, px, nullptr, nullptr, nullptr, nullptr, Cout, Nk, Mpix, Cout, 0, Nk, Nk, splits, ws, cg);
    const int64_t quads = (int64_t)Cout * Nk / 4;
    const int G = splitk_groups(quads, splits);
    splitk_reduce_k<T, kNone, false><<<(int)((quads * G + 255) / 256), 256, 0, s>>>(ws, splits, nullptr, pw, nullptr,
                                                                                   Cout, Nk, Nk, Nk, G);
    return;
  }
  gemm_lds_kernel<T, CF, false, false, kNone, false, false, false, 0, true><<<tiles, CF::NT, 0, s>>>(
      pdy, px, nullptr, pw, nullptr, nullptr, Cout, Nk, Mpix, Cout, 0, Nk, Nk, 1, nullptr, cg);
}
template <typename T>
void launch_conv_wgrad(const void* dy, const void* x, void* dW, int Mpix, int Cout, int Nk, const ConvGeom& cg,
                       int splits, float* ws, hipStream_t s) {
  if (Cout <= 128) launch_conv_wgrad_cfg<T, WG128>(dy, x, dW, Mpix, Cout, Nk, cg, splits, ws, s);
  else launch_conv_wgrad_cfg<T, W8>(dy, x, dW, Mpix, Cout, Nk, cg, splits, ws, s);
}

// tile by output channels: 512x64 for N <= 64, 256x128 for N <= 128, else 256x256 (split-K
// only there: the narrow tiles serve the large-M early layers)
inline int conv_tile_rows(int N) { return N <= 64 ? C64::BM : (N <= 128 ? C128::BM : W8::BM); }

template <typename T, int E>
int launch_conv(const void* xpad, const void* W, const void* bias, void* Y, int M, int N, int K, const ConvGeom& cg,
                int splits, float* ws, float* part, const float* kshift, hipStream_t s, const void* bnx = nullptr,
                const uint8_t* bnmask = nullptr, int beta = 0) {
  if (N <= 64) launch_conv_cfg<T, C64, E>(xpad, W, bias, Y, M, N, K, cg, 1, nullptr, part, kshift, s, bnx, bnmask, beta);
  else if (N <= 128)
    launch_conv_cfg<T, C128, E>(xpad, W, bias, Y, M, N, K, cg, 1, nullptr, part, kshift, s, bnx, bnmask, beta);
  else
    launch_conv_cfg<T, W8, E>(xpad, W, bias, Y, M, N, K, cg, part ? 1 : splits, ws, part, kshift, s, bnx, bnmask, beta);
  return 0;
}

}  // namespace
}  // namespace pra

// Implicit-GEMM convolution, channels-last, on the LDS-DMA MFMA kernel:
//   Y[N*Ho*Wo][Cout] = im2col(x) · Wkᵀ (+ bias, optional ReLU), zero padding P on H and W
// x is the input [N][H][W][C]; Wk the OHWI filter as a [Cout][KH*KW*C] matrix.
// Requires C % 64 == 0, Cout % 8 == 0 and x smaller than 2 GB (32-bit DMA offsets with the
// out-of-image sentinel above every valid one).
// splits > 1 (Cout > 128 only): split-K through the fp32 workspace ws [splits][M][Cout]
// (pra_conv_lds_splits gives the factor).
// part / kshift (optional, no split-K): BatchNorm statistics of Y per tile row,
// part [2][pra_conv_lds_stat_rows(M, Cout)][Cout] (see launch_conv_cfg).
extern "C" int pra_conv_lds_stat_rows(int M, int Cout) { return (M + pra::conv_tile_rows(Cout) - 1) / pra::conv_tile_rows(Cout); }

// pp (0 = C): the input's pixel pitch when it is narrower than C (see ConvGeom::PP): then
// KW == 1, P == 0, a tap row is C / pp adjacent pixels and Wo = (Wd - C / pp) / S + 1.
// bnx / bnmask (optional, a dgrad feeding BatchNorm(+ReLU)'s backward): Y = the product masked by
// the ReLU keep-bits bnmask ([M*Cout/8] bytes), part = per-tile sums of Y and of Y * (bnx - kshift)
// with bnx the BN input [M][Cout] and kshift its batch mean; needs part, kshift, no relu/bias/split.
// beta (bnx only): Y holds a pending gradient that is added to the product before the mask.
extern "C" int pra_conv_lds(const void* x, const void* W, const void* bias, void* Y, int Nimg, int H, int Wd,
                            int C, int Cout, int KH, int KW, int S, int P, int relu, int dtype, int splits, float* ws,
                            float* part, const float* kshift, int pp, hipStream_t s, const void* bnx = nullptr,
                            const uint8_t* bnmask = nullptr, int beta = 0) {
  if (pp <= 0) pp = C;
  if (bnx && (!bnmask || !part || !kshift || relu || bias || splits > 1)) return -1;
  if (C % 64 || Cout % 8 || KH <= 0 || KW <= 0 || S <= 0 || P < 0 || H <= 0 || Wd <= 0) return -1;
  if (pp != C && (pp % 8 || C % pp || KW != 1 || P != 0)) return -1;
  if (H >= 32768 || Wd >= 32768 || (long long)Nimg * H * Wd * pp * 2 >= (1ll << 31)) return -1;
  // (pp mode: a tap row is C / pp pixels wide)
  const int Ho = (H + 2 * P - KH) / S + 1, Wo = (pp != C ? Wd - C / pp : Wd + 2 * P - KW) / S + 1;
  if (Ho <= 0 || Wo <= 0) return -1;
  if (pp != C && (Wo - 1) * S + C / pp > Wd) return -1;
  const long long Mll = (long long)Nimg * Ho * Wo;
  if (Mll >= (1ll << 31)) return -1;
  const int M = (int)Mll, K = KH * KW * C;
  if (splits > 1 && (Cout <= 128 || !ws)) return -1;
  pra::ConvGeom cg{Ho, Wo, H, Wd, C, KW, S, P, pp};
  if (bnx) {
    if (dtype == pra::kBF16)
      return pra::launch_conv<pra::bf16, pra::kBnG>(x, W, nullptr, Y, M, Cout, K, cg, 1, nullptr, part, kshift, s, bnx,
                                                   bnmask, beta);
    if (dtype == pra::kF16)
      return pra::launch_conv<pra::f16, pra::kBnG>(x, W, nullptr, Y, M, Cout, K, cg, 1, nullptr, part, kshift, s, bnx,
                                                  bnmask, beta);
    return -1;
  }
  if (beta) return -1;
  if (dtype == pra::kBF16) return relu ? pra::launch_conv<pra::bf16, pra::kRelu>(x, W, bias, Y, M, Cout, K, cg, splits, ws, part, kshift, s)
                                  : pra::launch_conv<pra::bf16, pra::kNone>(x, W, bias, Y, M, Cout, K, cg, splits, ws, part, kshift, s);
  if (dtype == pra::kF16) return relu ? pra::launch_conv<pra::f16, pra::kRelu>(x, W, bias, Y, M, Cout, K, cg, splits, ws, part, kshift, s)
                                 : pra::launch_conv<pra::f16, pra::kNone>(x, W, bias, Y, M, Cout, K, cg, splits, ws, part, kshift, s);
  return -1;
}

// One sub-pixel phase of a stride-OS transposed convolution (the input gradient of a strided
// conv): dxp = conv_stride1(dy, Wp) over the Ho x Wo grid of dy with the phase's KHp x KWp taps
// at non-negative offsets (taps past the image edge read zeros), row (n, i, j) written to pixel
// (n, OS*i, OS*j) of dx_phase (dx + the phase's pixel offset, an (OS*Ho) x (OS*Wo) image).
// dy [Nimg][Ho][Wo][Co], Wp [Ci][KHp*KWp*Co]; Co % 64 == 0, Ci % 8 == 0. No split-K.
// bnx / bnmask / part / kshift: the kBnG epilogue as in pra_conv_lds (same phase offset applied
// to bnx and bnmask by the caller).
extern "C" int pra_conv_dgrad_phase(const void* dy, const void* Wp, void* dx_phase, int Nimg, int Ho, int Wo, int Co,
                                    int Ci, int KHp, int KWp, int OS, int dtype, float* part, const float* kshift,
                                    const void* bnx, const uint8_t* bnmask, hipStream_t s) {
  if (Co % 64 || Ci % 8 || KHp <= 0 || KWp <= 0 || OS < 2 || Ho <= 0 || Wo <= 0 || Ho >= 32768 || Wo >= 32768)
    return -1;
  if ((long long)Nimg * Ho * Wo * Co * 2 >= (1ll << 31) || (long long)Nimg * Ho * Wo * OS * OS * Ci * 2 >= (1ll << 31))
    return -1;
  if (bnx && (!bnmask || !part || !kshift)) return -1;
  const int M = Nimg * Ho * Wo, K = KHp * KWp * Co;
  pra::ConvGeom cg{Ho, Wo, Ho, Wo, Co, KWp, 1, 0, Co};
  cg.OS = OS;
  if (dtype == pra::kBF16)
    return bnx ? pra::launch_conv<pra::bf16, pra::kBnG>(dy, Wp, nullptr, dx_phase, M, Ci, K, cg, 1, nullptr, part, kshift,
                                                        s, bnx, bnmask)
               : pra::launch_conv<pra::bf16, pra::kNone>(dy, Wp, nullptr, dx_phase, M, Ci, K, cg, 1, nullptr, part,
                                                         kshift, s);
  if (dtype == pra::kF16)
    return bnx ? pra::launch_conv<pra::f16, pra::kBnG>(dy, Wp, nullptr, dx_phase, M, Ci, K, cg, 1, nullptr, part, kshift,
                                                       s, bnx, bnmask)
               : pra::launch_conv<pra::f16, pra::kNone>(dy, Wp, nullptr, dx_phase, M, Ci, K, cg, 1, nullptr, part, kshift,
                                                        s);
  return -1;
}

// Convolution weight gradient on the same kernel: dW (OHWI, [Cout][KH*KW*C]) from dy
// [N*Ho*Wo][Cout] and x [N][H][W][C]. Requires C % 64 == 0, Cout % 8 == 0, Cout >= 8, N*Ho*Wo
// % 64 == 0, x < 2 GB. splits > 1: fp32 workspace ws [splits][Cout][KH*KW*C].
// output-channel rows per weight-gradient tile (the caller sizes split-K from it)
extern "C" int pra_conv_wgrad_rows(int Cout) { return pra::conv_wgrad_rows(Cout); }
extern "C" int pra_conv_wgrad_lds(const void* dy, const void* x, void* dW, int Nimg, int H, int Wd, int C, int Cout,
                                  int KH, int KW, int S, int P, int dtype, int splits, float* ws, int pp,
                                  hipStream_t s) {
  if (pp <= 0) pp = C;
  if (C % 64 || Cout % 8 || Cout < 8 || KH <= 0 || KW <= 0 || S <= 0 || P < 0 || H <= 0 || Wd <= 0) return -1;
  if (pp != C && (pp % 8 || C % pp || KW != 1 || P != 0)) return -1;
  if (H >= 32768 || Wd >= 32768 || (long long)Nimg * H * Wd * pp * 2 >= (1ll << 31)) return -1;
  // (pp mode: a tap row is C / pp pixels wide)
  const int Ho = (H + 2 * P - KH) / S + 1, Wo = (pp != C ? Wd - C / pp : Wd + 2 * P - KW) / S + 1;
  if (Ho <= 0 || Wo <= 0) return -1;
  if (pp != C && (Wo - 1) * S + C / pp > Wd) return -1;
  const long long Mll = (long long)Nimg * Ho * Wo;
  if (Mll >= (1ll << 31) || Mll % 64 || (long long)Mll * Cout * 2 >= (1ll << 32)) return -1;
  if (splits > 1 && !ws) return -1;
  const int Nk = KH * KW * C;
  pra::ConvGeom cg{Ho, Wo, H, Wd, C, KW, S, P, pp};
  if (dtype == pra::kBF16) pra::launch_conv_wgrad<pra::bf16>(dy, x, dW, (int)Mll, Cout, Nk, cg, splits, ws, s);
  else if (dtype == pra::kF16) pra::launch_conv_wgrad<pra::f16>(dy, x, dW, (int)Mll, Cout, Nk, cg, splits, ws, s);
  else return -1;
  return 0;
}

// Split-K factor for an implicit-GEMM conv (1 for the narrow-tile configs, Cout <= 128)
extern "C" int pra_gemm_lds_splits(int M, int N, int K);
extern "C" int pra_conv_lds_splits(int M, int Cout, int K) { return Cout <= 128 ? 1 : pra_gemm_lds_splits(M, Cout, K); }

// Split-K factor for a problem: 1 unless the tile grid leaves CUs idle (fewer than ~224 tiles
// on a K loop of >= 16 steps); then the factor that minimises a simple time model:
//   rounds of 256 workgroups x (K-steps per split x 1.5 us + 3 us per-tile overhead)
//   + the fp32 partial round trip through HBM ((splits + 1) x M x N x 4 B at 5 TB/s),
// each split keeping >= 8 K-steps and the workspace <= 256 MB. The model reproduces the measured
// BERT wgrad times (profiles/r3g/gemm_bert_shapes.md: 768x768x16384 55 vs 53 us at 8 splits) and
// leaves every GPT-1.3B shape's factor unchanged; it lets few-tile / very-long-K products (BERT's
// 768x768 wgrad, ResNet's 1x1 weight gradients) fill the chip instead of 8 splits x few tiles.
extern "C" int pra_gemm_lds_splits(int M, int N, int K) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256), nk = K / 64;
  if (tiles >= 224 || nk < 16) return 1;
  int best = 1;
  double best_t = 1e30;
  for (int sp = 1; sp <= 256; ++sp) {
    if (nk / sp < 8) break;
    const double ws = (double)sp * M * N * 4.0;
    if (sp > 1 && ws > 256.0 * (1 << 20)) break;
    const double rounds = __builtin_ceil((double)tiles * sp / 256.0);
    const double per = __builtin_ceil((double)nk / sp) * 1.5 + 3.0;
    const double red = sp > 1 ? (double)(sp + 1) * M * N * 4.0 / 5e12 * 1e6 : 0.0;
    const double t = rounds * per + red;
    if (t < best_t - 1e-9) {
      best_t = t;
      best = sp;
    }
  }
  return best;
}

// layout: 0 = A[M][K]·B[K][N] (forward), 1 = A[M][K]·B[N][K]ᵀ (dgrad / NT), 2 = A[K][M]ᵀ·B[K][N] (wgrad).
// epi: 0 none, 1 gelu(erf), 2 gelu(tanh), 3 relu (Z receives the pre-activation if given),
//      4/5 dgelu(erf/tanh): C = acc * gelu'(Z) (Z required),
//      6/7 gelu(erf/tanh) with Z = gelu'(pre-activation) (x·W only, Z required),
//      8 C = acc * Z (dy·Wᵀ only, Z required: the saved derivative). colsum (optional, fp32
//      [ceil(M/256)][N]) receives per-tile column partial sums of the stored C.
// splits > 1: split-K through the fp32 workspace ws [splits][M][N] (not with dgelu/colsum).
// epi | 256: run the persistent kernel (gemm_pts.h) for this call when it takes the shape.
// Returns -1 (nothing launched) for shapes outside what the kernel assumes: K % 64, N % 8 and every
// leading dimension % 8 (16-B rows), M-contiguous operands need their MN extent >= 8.
extern "C" int pra_gemm_lds(int layout, const void* A, const void* B, const void* bias, void* C, void* Z, float* colsum,
                            int M, int N, int K, int lda, int ldb, int ldc, int ldz, int dtype, int epi, int beta,
                            int splits, float* ws, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || (K & 63) || (N & 7) || (lda & 7) || (ldb & 7) || (ldc & 7) || (ldz & 7)) return -1;
  if (layout == 2 && (M < 8 || (M & 7))) return -1;
  if ((layout == 0 || layout == 2) && N < 8) return -1;
  const int e = epi & 255;
  if (e >= 4 && e <= 8 && !Z) return -1;
  if (e > 8) return -1;
  if (splits > 1 && (!ws || e >= 4 || colsum || ldc != N)) return -1;
  // K-contiguous operands are addressed with 32-bit per-lane byte offsets from their base
  if ((layout == 0 || layout == 1) && (int64_t)M * lda * 2 >= (int64_t)1 << 32) return -1;
  if (layout == 1 && (int64_t)N * ldb * 2 >= (int64_t)1 << 32) return -1;
  if (splits < 1) splits = 1;
  struct ForcePts {  // scoped: the flag never outlives this call
    explicit ForcePts(bool on) { pra::g_force_pts = on; }
    ~ForcePts() { pra::g_force_pts = false; }
  } force_pts((epi & pra::kPersistBit) != 0 && splits == 1);
  epi &= ~pra::kPersistBit;
  if (dtype == pra::kBF16)
    return pra::launch_t<pra::bf16>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, splits, ws, s);
  if (dtype == pra::kF16)
    return pra::launch_t<pra::f16>(layout, A, B, bias, C, Z, colsum, M, N, K, lda, ldb, ldc, ldz, epi, beta, splits, ws, s);
  return -1;
}

extern "C" int pra_colsum_partials(const float* part, void* out, int P, int N, int dtype, hipStream_t s) {
  const int blocks = (N + 255) / 256;
  if (dtype == pra::kBF16) pra::colsum_partials_k<pra::bf16><<<blocks, 256, 0, s>>>(part, (pra::bf16*)out, P, N);
  else if (dtype == pra::kF16) pra::colsum_partials_k<pra::f16><<<blocks, 256, 0, s>>>(part, (pra::f16*)out, P, N);
  else if (dtype == pra::kF32) pra::colsum_partials_k<float><<<blocks, 256, 0, s>>>(part, (float*)out, P, N);
  else return -1;
  return 0;
}

extern "C" void pra_gemm_set_w4(int mask) { pra::g_w4_mask = mask; }
extern "C" void pra_gemm_set_pts(int mask) { pra::g_pts_mask = mask; }
extern "C" int pra_gemm_get_pts() { return pra::pts_mask(); }
extern "C" int pra_gemm_get_w4() { return pra::w4_mask(); }
