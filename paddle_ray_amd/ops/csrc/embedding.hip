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

// Long runs (a position or token-type id repeated across the whole batch: one run of 16K rows
// for BERT's token types) would leave ONE wave summing the whole run. The two-pass form cuts
// every run at fixed kSeg-aligned positions: pass 1 has one wave per segment (a piece of a run
// inside one aligned block) sum its <= kSeg rows; a run that fits in its block is finished
// there (the common case: word ids), otherwise the partial goes to the scratch slot A[b] (the
// segment starting the aligned block b) or B[b] (the run's first segment, when the run goes on
// past its block). Pass 2 has one wave per block: if the run started in block b continues past
// it, the wave adds B[b] and the A slots of the blocks the run covers and writes dW. Still
// deterministic, no float atomics.
constexpr int kSeg = 32;

template <typename TG, typename TW, int NC>
__global__ void __launch_bounds__(kEmbWaves * 64) emb_bwd_seg_k(const int64_t* __restrict__ sorted_ids,
                                                                const int64_t* __restrict__ perm,
                                                                const TG* __restrict__ dy, TW* __restrict__ dw,
                                                                float* __restrict__ ws, int64_t n, int D, int64_t V,
                                                                int64_t pad, int accumulate) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kEmbWaves + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t id = sorted_ids[i];
  const bool run_start = i == 0 || sorted_ids[i - 1] != id;
  if (!run_start && i % kSeg != 0) return;  // not a segment start
  if (id < 0 || id >= V || id == pad) return;
  float acc[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[c][k] = 0.f;
  int64_t j = i;
  do {
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
    ++j;
  } while (j < n && j % kSeg != 0 && sorted_ids[j] == id);
  const bool goes_on = j < n && sorted_ids[j] == id;  // the run continues into the next block
  const int64_t nb = (n + kSeg - 1) / kSeg;
  float* slot = nullptr;
  if (!run_start) slot = ws + (i / kSeg) * (int64_t)D;                 // A[b]
  else if (goes_on) slot = ws + (nb + i / kSeg) * (int64_t)D;          // B[b]
  if (slot) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < D) store8<float>(slot + col, acc[c]);
    }
    return;
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

template <typename TW, int NC>
__global__ void __launch_bounds__(kEmbWaves * 64) emb_bwd_fin_k(const int64_t* __restrict__ sorted_ids,
                                                                TW* __restrict__ dw, const float* __restrict__ ws,
                                                                int64_t n, int D, int64_t V, int64_t pad,
                                                                int accumulate) {
  const int lane = threadIdx.x & 63;
  const int64_t nb = (n + kSeg - 1) / kSeg;
  const int64_t b = (int64_t)blockIdx.x * kEmbWaves + (threadIdx.x >> 6);
  if (b >= nb) return;
  const int64_t e = min(n, (b + 1) * kSeg) - 1;  // last position of block b
  const int64_t id = sorted_ids[e];
  if (e + 1 >= n || sorted_ids[e + 1] != id) return;      // its run ends inside block b
  if (b > 0 && sorted_ids[b * kSeg - 1] == id) return;      // ... or started before block b
  if (id < 0 || id >= V || id == pad) return;
  float acc[NC][8];
  const float* src = ws + (nb + b) * (int64_t)D;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < D) load8<float>(src + col, acc[c]);
  }
  for (int64_t k = b + 1; k < nb && sorted_ids[k * kSeg] == id; ++k) {
    const float* a = ws + k * (int64_t)D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < D) {
        float v[8];
        load8<float>(a + col, v);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[c][q] += v[q];
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
        for (int q = 0; q < 8; ++q) acc[c][q] += old[q];
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

// ws: scratch of 2 * ceil(n / 32) * D floats for the segmented two-pass form (long runs split
// over many waves); nullptr = one wave per run.
int pra_embedding_bwd(const int64_t* sorted_ids, const int64_t* perm, const void* dy, void* dw, int64_t n, int D,
                      int64_t V, int64_t pad, int dt_dy, int dt_w, int accumulate, float* ws, hipStream_t s) {
  if (D % 8 != 0 || D > 8 * 512) return -1;
  if (n == 0) return 0;
  const dim3 grid((unsigned)((n + kEmbWaves - 1) / kEmbWaves));
  const int nc = (D + 511) / 512;
  const int64_t nb = (n + kSeg - 1) / kSeg;
  const dim3 gridb((unsigned)((nb + kEmbWaves - 1) / kEmbWaves));
#define PRA_EMB_SEG(TG, TW, NC)                                                                                  \
  do {                                                                                                           \
    hipLaunchKernelGGL((emb_bwd_seg_k<TG, TW, NC>), grid, dim3(kEmbWaves * 64), 0, s, sorted_ids, perm,          \
                       (const TG*)dy, (TW*)dw, ws, n, D, V, pad, accumulate);                                    \
    hipLaunchKernelGGL((emb_bwd_fin_k<TW, NC>), gridb, dim3(kEmbWaves * 64), 0, s, sorted_ids, (TW*)dw,          \
                       (const float*)ws, n, D, V, pad, accumulate);                                              \
  } while (0)
#define PRA_EMB_BWD(TG, TW)                                                                                    \
  do {                                                                                                         \
    if (ws) {                                                                                                  \
      if (nc <= 1) PRA_EMB_SEG(TG, TW, 1);                                                                     \
      else if (nc <= 2) PRA_EMB_SEG(TG, TW, 2);                                                                \
      else if (nc <= 4) PRA_EMB_SEG(TG, TW, 4);                                                                \
      else PRA_EMB_SEG(TG, TW, 8);                                                                             \
      break;                                                                                                   \
    }                                                                                                          \
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
#undef PRA_EMB_SEG
  return 0;
}
}
