// Sharded LAMB on one rank's slice of the flat parameter space (DistributedFusedLamb; parity:
// paddle/fluid/operators/optimizers/distributed_fused_lamb_op.cu -- moments and fp32 master
// weights sharded 1/nranks, per-parameter trust ratio ||w|| / ||r|| over the WHOLE parameter).
//
// The shard is contiguous (FlatGroup layout), so no multi-tensor table is needed: a block table
// cuts it into pieces that never cross a parameter boundary, piece b = {param index, lo, hi}.
//   stage 1: g' = g * gscale (1/nranks, clip coefficient from the device), m / v updated in
//            place, r = m^ / (sqrt(v^) + eps) + wd_p * w stored in a fp32 scratch shard, and the
//            per-parameter partial sums of w^2 and r^2 (one float atomic per block each);
//   (host)   the [2][P] partial sums are all-reduced across ranks;
//   stage 2: w -= lr * trust_p * r with trust_p = ||w_p|| / ||r_p|| (1 when either is 0); the
//            updated master goes to the shard of the parameter buffer in the parameter's dtype
//            (what the all-gather then distributes).
#include "common.h"

namespace pra {
namespace {

__device__ __forceinline__ float ld_t(const void* p, int64_t i, int dt) {
  if (dt == kF32) return static_cast<const float*>(p)[i];
  if (dt == kBF16) return bf2f(static_cast<const uint16_t*>(p)[i]);
  return (float)static_cast<const _Float16*>(p)[i];
}
__device__ __forceinline__ void st_t(void* p, int64_t i, int dt, float v) {
  if (dt == kF32) static_cast<float*>(p)[i] = v;
  else if (dt == kBF16) static_cast<uint16_t*>(p)[i] = f2bf(v);
  else static_cast<_Float16*>(p)[i] = (_Float16)v;
}

__global__ void __launch_bounds__(256) lamb_stage1_k(const int64_t* __restrict__ pieces, const void* __restrict__ g,
                                                     int gdt, const float* __restrict__ w, float* __restrict__ m,
                                                     float* __restrict__ v, float* __restrict__ r,
                                                     const float* __restrict__ wd, float* __restrict__ norms, int P,
                                                     float b1, float b2, float eps, float rbc1, float rbc2,
                                                     float gscale, const float* __restrict__ gscale_ptr) {
  __shared__ float red[16];
  if (gscale_ptr) gscale *= *gscale_ptr;
  const int64_t p = pieces[3 * blockIdx.x], lo = pieces[3 * blockIdx.x + 1], hi = pieces[3 * blockIdx.x + 2];
  const float wdp = wd[p];
  float sw = 0.f, sr = 0.f;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const float gi = ld_t(g, i, gdt) * gscale;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float wi = w[i];
    const float ri = mi * rbc1 / (sqrtf(vi * rbc2) + eps) + wdp * wi;
    r[i] = ri;
    sw += wi * wi;
    sr += ri * ri;
  }
  sw = block_sum(sw, red);
  sr = block_sum(sr, red);
  if (threadIdx.x == 0) {
    atomicAdd(norms + p, sw);
    atomicAdd(norms + P + p, sr);
  }
}

__global__ void __launch_bounds__(256) lamb_stage2_k(const int64_t* __restrict__ pieces, float* __restrict__ w,
                                                     const float* __restrict__ r, const float* __restrict__ norms,
                                                     int P, float lr, void* __restrict__ pout, int pdt) {
  const int64_t p = pieces[3 * blockIdx.x], lo = pieces[3 * blockIdx.x + 1], hi = pieces[3 * blockIdx.x + 2];
  const float wn = sqrtf(norms[p]), rn = sqrtf(norms[P + p]);
  const float trust = (wn > 0.f && rn > 0.f) ? wn / rn : 1.f;
  const float step = lr * trust;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const float wi = w[i] - step * r[i];
    w[i] = wi;
    if (pout) st_t(pout, i, pdt, wi);
  }
}

}  // namespace
}  // namespace pra

extern "C" void pra_lamb_shard_stage1(const int64_t* pieces, int npieces, const void* g, int gdt, const float* w,
                                      float* m, float* v, float* r, const float* wd, float* norms, int P, float b1,
                                      float b2, float eps, float bc1, float bc2, float gscale,
                                      const float* gscale_ptr, hipStream_t s) {
  if (npieces <= 0) return;
  hipLaunchKernelGGL(pra::lamb_stage1_k, dim3(npieces), dim3(256), 0, s, pieces, g, gdt, w, m, v, r, wd, norms, P,
                     b1, b2, eps, 1.f / bc1, 1.f / bc2, gscale, gscale_ptr);
}

extern "C" void pra_lamb_shard_stage2(const int64_t* pieces, int npieces, float* w, const float* r,
                                      const float* norms, int P, float lr, void* pout, int pdt, hipStream_t s) {
  if (npieces <= 0) return;
  hipLaunchKernelGGL(pra::lamb_stage2_k, dim3(npieces), dim3(256), 0, s, pieces, w, r, norms, P, lr, pout, pdt);
}
