// Single-token (decode-phase) multi-head attention over a KV cache, for gfx950.
//
// Parity: the reference's masked multihead attention decoder kernel behind
// fused_multi_transformer (paddle/fluid/operators/fused/fused_multi_transformer_op.cu.h,
// mmha_launch_kernel): q·K over the cache positions [0, t], additive mask, softmax, ·V, and the
// new token's K/V written into the cache at position t.
//
// MI355X design (memory bound: every step streams the whole K/V cache once):
//  * split-K "flash decoding": grid (splits, heads, batch); each workgroup owns a contiguous
//    key range and keeps an online-softmax (max, sum, acc[D]) in registers; a second tiny
//    kernel merges the splits. Splits are sized so a decode step launches >= ~1024
//    workgroups (4 per CU) even at batch 1.
//  * G = D/8 lanes per key: each lane holds 8 of the D dims, so one key row (D*2 bytes) is
//    read by G consecutive lanes as 16-byte vectors — fully coalesced — and a 64-wide wave
//    works on 64/G keys at once. q·k is reduced over the G lanes with xor-shuffles that
//    never leave the group.
//  * two keys per lane-group per iteration are loaded before any math so >= 4 16-byte loads
//    per lane are in flight.
//  * the new token's K/V never round-trips through the cache: the workgroup that owns
//    position t uses them from the qkv buffer and writes them into the cache (vector stores).
#include "common.h"

namespace pra {
namespace {

constexpr int kWaves = 4;

template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// merge (m2, l2, a2) into (m, l, a)
template <int N>
__device__ __forceinline__ void merge(float& m, float& l, float* a, float m2, float l2, const float* a2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;
  const float c1 = (m == -INFINITY) ? 0.f : __expf(m - M);
  const float c2 = (m2 == -INFINITY) ? 0.f : __expf(m2 - M);
  l = l * c1 + l2 * c2;
#pragma unroll
  for (int i = 0; i < N; ++i) a[i] = a[i] * c1 + a2[i] * c2;
  m = M;
}

template <typename T, int D>
__global__ void __launch_bounds__(kWaves * 64) mmha_split_k(
    const T* __restrict__ qkv,      // [B, 3, H, D] (bias already added)
    T* __restrict__ cache,          // [2, B, H, L, D]
    const float* __restrict__ mask, // [B, mask_len] additive, or null
    float* __restrict__ ws_ml,      // [B, H, S, 2]
    float* __restrict__ ws_acc,     // [B, H, S, D]
    T* __restrict__ out,            // [B, H, D] (used when splits == 1)
    int B, int H, int L, int t_host, const int* __restrict__ t_dev, int keys_per_split, int mask_len,
    float scale) {
  // t_dev (HIP-graph decode loops): the position comes from device memory, so one captured
  // graph serves every step; an out-of-range position writes nothing and outputs zeros
  const int t = t_dev ? t_dev[0] : t_host;
  constexpr int G = D / 8;            // lanes per key
  constexpr int KPW = 64 / G;         // keys per wave per sub-step
  const int split = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int splits = gridDim.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int gl = lane % G, grp = lane / G;
  const bool t_ok = t >= 0 && t < L && !(mask && mask_len < t + 1);
  const int lo = split * keys_per_split;
  const int hi = t_ok ? min(t + 1, lo + keys_per_split) : lo;

  const size_t BH = (size_t)B * H;
  const T* qrow = qkv + ((size_t)b * 3 * H + h) * D;
  const T* knew = qkv + ((size_t)b * 3 * H + H + h) * D;
  const T* vnew = qkv + ((size_t)b * 3 * H + 2 * H + h) * D;
  T* kc = cache + ((size_t)b * H + h) * (size_t)L * D;
  T* vc = cache + (BH + (size_t)b * H + h) * (size_t)L * D;

  if (t_ok && t >= lo && t < hi && wave == 0 && grp == 0) {  // append the new token to the cache
    float kv[8];
    load8<T>(knew + gl * 8, kv);
    store8<T>(kc + (size_t)t * D + gl * 8, kv);
    load8<T>(vnew + gl * 8, kv);
    store8<T>(vc + (size_t)t * D + gl * 8, kv);
  }

  float q[8];
  load8<T>(qrow + gl * 8, q);
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] *= scale;

  float m = -INFINITY, l = 0.f, acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;

  const float* mrow = mask ? mask + (size_t)b * mask_len : nullptr;
  constexpr int STEP = kWaves * KPW * 2;
  for (int base = lo; base < hi; base += STEP) {
    int key[2];
    float kx[2][8], vx[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      key[u] = base + (u * kWaves + wave) * KPW + grp;
      const int kk = key[u] < hi ? key[u] : lo;
      const T* kp = (kk == t) ? knew : kc + (size_t)kk * D;
      const T* vp = (kk == t) ? vnew : vc + (size_t)kk * D;
      load8<T>(kp + gl * 8, kx[u]);
      load8<T>(vp + gl * 8, vx[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s += q[i] * kx[u][i];
      s = group_sum<G>(s);
      if (key[u] >= hi) continue;
      if (mrow) s += mrow[key[u]];
      const float mn = fmaxf(m, s);
      if (mn == -INFINITY) continue;  // fully masked so far
      const float c = (m == -INFINITY) ? 0.f : __expf(m - mn);
      const float p = __expf(s - mn);
      l = l * c + p;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = acc[i] * c + p * vx[u][i];
      m = mn;
    }
  }

  // merge the KPW key groups of this wave (lanes gl, gl+G, ...)
#pragma unroll
  for (int o = G; o < 64; o <<= 1) {
    const float m2 = __shfl_xor(m, o, 64), l2 = __shfl_xor(l, o, 64);
    float a2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a2[i] = __shfl_xor(acc[i], o, 64);
    merge<8>(m, l, acc, m2, l2, a2);
  }
  // merge the waves through LDS
  __shared__ float s_ml[kWaves][2];
  __shared__ float s_acc[kWaves][D];
  if (grp == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s_acc[wave][gl * 8 + i] = acc[i];
    if (gl == 0) { s_ml[wave][0] = m; s_ml[wave][1] = l; }
  }
  __syncthreads();
  if (wave != 0 || grp != 0) return;
  for (int w = 1; w < kWaves; ++w) merge<8>(m, l, acc, s_ml[w][0], s_ml[w][1], &s_acc[w][gl * 8]);
  if (splits == 1) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= inv;
    store8<T>(out + ((size_t)b * H + h) * D + gl * 8, acc);
    return;
  }
  const size_t w = ((size_t)b * H + h) * splits + split;
  float* wa = ws_acc + w * D + gl * 8;
  *reinterpret_cast<float4*>(wa) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(wa + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  if (gl == 0) *reinterpret_cast<float2*>(ws_ml + w * 2) = make_float2(m, l);
}

template <typename T, int D>
__global__ void __launch_bounds__(D) mmha_combine_k(const float* __restrict__ ws_ml, const float* __restrict__ ws_acc,
                                                    T* __restrict__ out, int splits) {
  const int h = blockIdx.x, b = blockIdx.y, H = gridDim.x, d = threadIdx.x;
  const size_t w0 = ((size_t)b * H + h) * splits;
  float M = -INFINITY;
  for (int s = 0; s < splits; ++s) M = fmaxf(M, ws_ml[(w0 + s) * 2]);
  float num = 0.f, den = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < splits; ++s) {
      const float ms = ws_ml[(w0 + s) * 2];
      if (ms == -INFINITY) continue;
      const float c = __expf(ms - M);
      den += ws_ml[(w0 + s) * 2 + 1] * c;
      num += ws_acc[(w0 + s) * D + d] * c;
    }
  }
  out[((size_t)b * H + h) * D + d] = Cvt<T>::from(den > 0.f ? num / den : 0.f);
}

template <typename T, int D>
int launch(const void* qkv, void* cache, const float* mask, float* ws, void* out, int B, int H, int L, int t,
           const int* t_dev, int splits, int mask_len, float scale, hipStream_t s) {
  const int keys = t_dev ? L : t + 1;  // device position: splits cover the whole cache
  const int per = (keys + splits - 1) / splits;
  float* ws_ml = ws;
  float* ws_acc = ws + (((size_t)B * H * splits * 2 + 3) / 4) * 4;  // 16-B aligned
  hipLaunchKernelGGL((mmha_split_k<T, D>), dim3(splits, H, B), dim3(kWaves * 64), 0, s, (const T*)qkv, (T*)cache,
                     mask, ws_ml, ws_acc, (T*)out, B, H, L, t, t_dev, per, mask_len, scale);
  if (splits > 1)
    hipLaunchKernelGGL((mmha_combine_k<T, D>), dim3(H, B), dim3(D), 0, s, ws_ml, ws_acc, (T*)out, splits);
  return 0;
}

}  // namespace
}  // namespace pra

using namespace pra;

extern "C" {
// workgroups per decode step: aim for >= 1024 (4 per CU) with >= 64 keys per split
int pra_mmha_splits(int B, int H, int t) {
  const int keys = t + 1;
  int want = (1024 + B * H - 1) / (B * H);
  int cap = (keys + 63) / 64;
  int s = want < cap ? want : cap;
  if (s < 1) s = 1;
  if (s > 256) s = 256;
  return s;
}

// ws: fp32 workspace of B*H*splits*(2 + D) + 4 floats (unused when splits == 1)
int pra_mmha_decode(const void* qkv, void* cache, const float* mask, float* ws, void* out, int B, int H, int L,
                    int D, int t, const int* t_dev, int splits, int mask_len, float scale, int dt, hipStream_t s) {
  if (splits < 1) return -1;
  if (!t_dev && (t < 0 || t >= L || (mask && mask_len < t + 1))) return -1;
#define PRA_MMHA(TT)                                                                                          \
  switch (D) {                                                                                                \
    case 64: return launch<TT, 64>(qkv, cache, mask, ws, out, B, H, L, t, t_dev, splits, mask_len, scale, s);        \
    case 128: return launch<TT, 128>(qkv, cache, mask, ws, out, B, H, L, t, t_dev, splits, mask_len, scale, s);      \
    case 256: return launch<TT, 256>(qkv, cache, mask, ws, out, B, H, L, t, t_dev, splits, mask_len, scale, s);      \
    default: return -1;                                                                                       \
  }
  if (dt == kBF16) { PRA_MMHA(bf16) }
  if (dt == kF16) { PRA_MMHA(f16) }
  if (dt == kF32) { PRA_MMHA(float) }
#undef PRA_MMHA
  return -1;
}
}
