// Embedding lookup forward + weight-gradient for gfx950.
//
// Parity: paddle/phi/kernels/gpu/embedding_kernel.cu, embedding_grad_kernel.cu
// (lookup_table_v2). Rows of the table are D contiguous elements, D % 8 == 0, so every
// access is a 16-byte vector and one 64-lane wave moves 1 KB of a row per instruction.
//
// forward : out[t, :] = W[ids[t], :]; ids outside [0, V) or == padding_idx give zeros
//           (never an out-of-bounds read).
// backward: deterministic segmented sum without float atomics. The caller sorts the ids
//           (stable) once; one wave per run of equal ids sums the run's dy rows in fp32
//           registers and adds the result into dW's row in place (read-modify-write of the
//           existing gradient, so the optimizer's flat grad buffer is accumulated directly and
//           no dense [V, D] temporary or extra add pass exists). Runs own disjoint rows: no
//           races.
#include "common.h"

namespace pra {

constexpr int kEmbWaves = 4;  // waves per workgroup

template <typename T>
__global__ void __launch_bounds__(kEmbWaves * 64) emb_fwd_k(const int64_t* __restrict__ ids,
                                                            const T* __restrict__ w, T* __restrict__ out,
                                                            int64_t n, int D, int64_t V, int64_t pad) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kEmbWaves + (threadIdx.x >> 6);
  if (row >= n) return;
  const int64_t id = ids[row];
  const bool ok = id >= 0 && id < V && id != pad;
  T* o = out + row * D;
  const T* src = w + (ok ? id : 0) * (int64_t)D;
  for (int c = lane * 8; c < D; c += 64 * 8) {
    uint4 v = ok ? *reinterpret_cast<const uint4*>(src + c) : make_uint4(0, 0, 0, 0);
    if (sizeof(T) == 4) {  // fp32 rows: two 16-B vectors per 8 elements
      uint4 v2 = ok ? *reinterpret_cast<const uint4*>(src + c + 4) : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(o + c + 4) = v2;
    }
    *reinterpret_cast<uint4*>(o + c) = v;
  }
}

// sorted_ids[i], perm[i]: position i of the stable sort of ids; one wave per run start.
// NC = number of 512-element column chunks held in registers (D <= 512 * NC).
template <typename TG, typename TW, int NC>
__global__ void __launch_bounds__(kEmbWaves * 64) emb_bwd_k(const int64_t* __restrict__ sorted_ids,
                                                            const int64_t* __restrict__ perm,
                                                            const TG* __restrict__ dy, TW* __restrict__ dw,
                                                            int64_t n, int D, int64_t V, int64_t pad,
                                                            int accumulate) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kEmbWaves + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t id = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == id) return;  // not a run start
  if (id < 0 || id >= V || id == pad) return;
  float acc[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[c][k] = 0.f;
  for (int64_t j = i; j < n && sorted_ids[j] == id; ++j) {
    const TG* src = dy + perm[j] * (int64_t)D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < D) {
        float v[8];
        load8<TG>(src + col, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[c][k] += v[k];
      }
    }
  }
  TW* dst = dw + id * (int64_t)D;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < D) {
      if (accumulate) {
        float old[8];
        load8<TW>(dst + col, old);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[c][k] += old[k];
      }
      store8<TW>(dst + col, acc[c]);
    }
  }
}

}  // namespace pra

using namespace pra;

extern "C" {
int pra_embedding_fwd(const int64_t* ids, const void* w, void* out, int64_t n, int D, int64_t V, int64_t pad, int dt,
                      hipStream_t s) {
  if (D % 8 != 0) return -1;
  if (n == 0) return 0;
  const dim3 grid((unsigned)((n + kEmbWaves - 1) / kEmbWaves));
  switch (dt) {
    case kF32: hipLaunchKernelGGL((emb_fwd_k<float>), grid, dim3(kEmbWaves * 64), 0, s, ids, (const float*)w,
                                  (float*)out, n, D, V, pad); break;
    case kBF16: hipLaunchKernelGGL((emb_fwd_k<bf16>), grid, dim3(kEmbWaves * 64), 0, s, ids, (const bf16*)w,
                                   (bf16*)out, n, D, V, pad); break;
    case kF16: hipLaunchKernelGGL((emb_fwd_k<f16>), grid, dim3(kEmbWaves * 64), 0, s, ids, (const f16*)w,
                                  (f16*)out, n, D, V, pad); break;
    default: return -1;
  }
  return 0;
}

int pra_embedding_bwd(const int64_t* sorted_ids, const int64_t* perm, const void* dy, void* dw, int64_t n, int D,
                      int64_t V, int64_t pad, int dt_dy, int dt_w, int accumulate, hipStream_t s) {
  if (D % 8 != 0 || D > 8 * 512) return -1;
  if (n == 0) return 0;
  const dim3 grid((unsigned)((n + kEmbWaves - 1) / kEmbWaves));
  const int nc = (D + 511) / 512;
#define PRA_EMB_BWD(TG, TW)                                                                                    \
  do {                                                                                                         \
    if (nc <= 1) hipLaunchKernelGGL((emb_bwd_k<TG, TW, 1>), grid, dim3(kEmbWaves * 64), 0, s, sorted_ids, perm, \
                                    (const TG*)dy, (TW*)dw, n, D, V, pad, accumulate);                         \
    else if (nc <= 2) hipLaunchKernelGGL((emb_bwd_k<TG, TW, 2>), grid, dim3(kEmbWaves * 64), 0, s, sorted_ids,  \
                                         perm, (const TG*)dy, (TW*)dw, n, D, V, pad, accumulate);              \
    else if (nc <= 4) hipLaunchKernelGGL((emb_bwd_k<TG, TW, 4>), grid, dim3(kEmbWaves * 64), 0, s, sorted_ids,  \
                                         perm, (const TG*)dy, (TW*)dw, n, D, V, pad, accumulate);              \
    else hipLaunchKernelGGL((emb_bwd_k<TG, TW, 8>), grid, dim3(kEmbWaves * 64), 0, s, sorted_ids, perm,         \
                            (const TG*)dy, (TW*)dw, n, D, V, pad, accumulate);                                 \
  } while (0)
  if (dt_dy == kBF16 && dt_w == kBF16) PRA_EMB_BWD(bf16, bf16);
  else if (dt_dy == kBF16 && dt_w == kF32) PRA_EMB_BWD(bf16, float);
  else if (dt_dy == kF32 && dt_w == kF32) PRA_EMB_BWD(float, float);
  else if (dt_dy == kF16 && dt_w == kF16) PRA_EMB_BWD(f16, f16);
  else if (dt_dy == kF16 && dt_w == kF32) PRA_EMB_BWD(f16, float);
  else return -1;
#undef PRA_EMB_BWD
  return 0;
}
}
