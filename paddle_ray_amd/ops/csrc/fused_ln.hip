// Fused residual-add + dropout (+bias) + LayerNorm, forward and backward, for gfx950.
//
//   r = x + dropout(h + hbias)        (h == nullptr: r = x, no dropout)
//   y = LayerNorm(r) * w + b
//
// One WAVE per row (cols <= 4096, cols % 8 == 0): the row lives in registers
// (C chunks of 8 per lane), all reductions are wave shuffles (no LDS, no
// barriers), 16-byte vector loads/stores. Dropout uses a counter-based hash
// RNG keyed by (seed, offset, element index), so backward REGENERATES the mask
// instead of reading a stored one (no [tokens, hidden] mask tensor in HBM).
// Backward accumulates dW/dB/dBias partials per workgroup in registers and
// reduces the 4 waves through LDS; `colsum16` folds the [nblk, cols] partials
// with 16 columns x 16 row-slices per workgroup (deterministic, no atomics).
//
// Parity: paddle/fluid/operators/fused/fused_dropout_helper.h,
// fused_layernorm_residual_dropout_bias.h (FusedBiasDropoutResidualLayerNorm).
#include "common.h"
#include <stdlib.h>

namespace pra {

template <typename T> __device__ __forceinline__ void round8(float* v) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = Cvt<T>::to(Cvt<T>::from(v[i]));
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
// 16-bit uniforms for elements [i, i+1] of the flat tensor
__device__ __forceinline__ uint32_t rng_pair(uint64_t seed, uint64_t offset, uint64_t i) {
  uint64_t c = (i >> 1) + offset;
  uint32_t a = mix32((uint32_t)c ^ (uint32_t)seed);
  return mix32(a ^ (uint32_t)(c >> 32) ^ (uint32_t)(seed >> 32) ^ 0x9e3779b9U);
}
// keep-mask bits for 8 consecutive elements starting at flat index i (i % 8 == 0)
__device__ __forceinline__ void keep8(uint64_t seed, uint64_t offset, uint64_t i, uint32_t thr, bool* k) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t r = rng_pair(seed, offset, i + 2 * j);
    k[2 * j] = (r & 0xffffu) >= thr;
    k[2 * j + 1] = (r >> 16) >= thr;
  }
}

template <typename T, typename W, int C>
__global__ void __launch_bounds__(256) adl_fwd_k(const T* __restrict__ x, const T* __restrict__ h,
                                                 const T* __restrict__ hbias, const W* __restrict__ w,
                                                 const W* __restrict__ b, T* __restrict__ r_out,
                                                 T* __restrict__ y, float* __restrict__ mean,
                                                 float* __restrict__ rstd, int rows, int cols, float eps,
                                                 uint32_t thr, float scale, uint64_t seed, uint64_t offset,
                                                 const uint64_t* __restrict__ dseq) {
  if (dseq) seed ^= *dseq * 0x9E3779B97F4A7C15ull;  // graph replays: device step counter (see graph_seq)
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t base = (size_t)row * cols;
  float v[C][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int idx = (c * 64 + lane) * 8;
    if (idx < cols) {
      load8<T>(x + base + idx, v[c]);
      if (h) {
        float hv[8], bv[8];
        load8<T>(h + base + idx, hv);
        if (hbias) load8<T>(hbias + idx, bv);
        bool k[8];
        if (thr) keep8(seed, offset, base + idx, thr, k);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float t = hv[i] + (hbias ? bv[i] : 0.f);
          if (thr) t = k[i] ? t * scale : 0.f;
          v[c][i] += t;
        }
        if (r_out) {
          store8<T>(r_out + base + idx, v[c]);
          round8<T>(v[c]);  // stats of the ROUNDED residual, exactly what backward re-reads
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
    }
  }
  const float mu = wave_sum(s) / cols;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int idx = (c * 64 + lane) * 8;
    if (idx < cols) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { float d = v[c][i] - mu; ss += d * d; }
    }
  }
  const float rs = rsqrtf(wave_sum(ss) / cols + eps);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int idx = (c * 64 + lane) * 8;
    if (idx < cols) {
      float wv[8], bv[8], o[8];
      if (w) load8<W>(w + idx, wv); else {
#pragma unroll
        for (int i = 0; i < 8; ++i) wv[i] = 1.f;
      }
      if (b) load8<W>(b + idx, bv); else {
#pragma unroll
        for (int i = 0; i < 8; ++i) bv[i] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mu) * rs * wv[i] + bv[i];
      store8<T>(y + base + idx, o);
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

// dy: grad of y; dr_out: extra grad arriving at r from its other consumer (may be null)
// outputs: dr_in (= total grad of r = grad of x), dh (= dr_in * keep * scale) if h path
// TWO = false: one pass per row, xh / dy*w / dr_out held in registers across the row reductions
// (248 VGPRs: 2 waves per SIMD). TWO = true: the row is read twice -- pass 1 only accumulates
// the row sums and the dW / dB partials, pass 2 re-reads r and dy (L2-resident: the wave just
// read them) with dr_out and writes the outputs -- so nothing row-sized stays live across the
// reductions and the kernel fits 3 waves per SIMD (more HBM reads in flight per CU).
template <typename T, typename W, int C, bool TWO>
__device__ __forceinline__ void adl_bwd_body(const T* __restrict__ dy, const T* __restrict__ dr_out,
                                             const T* __restrict__ r, const W* __restrict__ w,
                                             const float* __restrict__ mean, const float* __restrict__ rstd,
                                             T* __restrict__ dr_in, T* __restrict__ dh,
                                             float* __restrict__ pw, float* __restrict__ pb,
                                             float* __restrict__ pbias, int rows, int cols, uint32_t thr,
                                             float scale, uint64_t seed, uint64_t offset,
                                             const uint64_t* __restrict__ dseq) {
  if (dseq) seed ^= *dseq * 0x9E3779B97F4A7C15ull;
  extern __shared__ __attribute__((aligned(16))) float red_lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float aw[C][8], ab[C][8], ah[C][8];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) { aw[c][i] = 0.f; ab[c][i] = 0.f; ah[c][i] = 0.f; }
  for (int row = blockIdx.x * 4 + wid; row < rows; row += gridDim.x * 4) {
    const size_t base = (size_t)row * cols;
    const float mu = mean[row], rs = rstd[row];
    float xh[TWO ? 1 : C][8], g[TWO ? 1 : C][8], e[TWO ? 1 : C][8];
    // (one pass) the residual's incoming grad is loaded with r / dy (not after the row
    // reductions): one memory round trip per row instead of two. The LN weight is re-read per
    // row (L1/L2-resident) instead of pinned in registers, which pays for e[][].
    if (!TWO && dr_out) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const int idx = (c * 64 + lane) * 8;
        if (idx < cols) load8<T>(dr_out + base + idx, e[c]);
      }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < cols) {
        float rv[8], dv[8], wv[8];
        load8<T>(r + base + idx, rv);
        load8<T>(dy + base + idx, dv);
        if (w) load8<W>(w + idx, wv);
        else {
#pragma unroll
          for (int i = 0; i < 8; ++i) wv[i] = 1.f;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float x_ = (rv[i] - mu) * rs, g_ = dv[i] * wv[i];
          if constexpr (!TWO) { xh[c][i] = x_; g[c][i] = g_; }
          s1 += g_ * x_;
          s2 += g_;
          aw[c][i] += dv[i] * x_;
          ab[c][i] += dv[i];
        }
      }
    }
    const float c1 = wave_sum(s1) / cols, c2 = wave_sum(s2) / cols;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < cols) {
        float o[8];
        if constexpr (TWO) {
          float rv[8], dv[8], wv[8], ev[8];
          load8<T>(r + base + idx, rv);
          load8<T>(dy + base + idx, dv);
          if (dr_out) load8<T>(dr_out + base + idx, ev);
          if (w) load8<W>(w + idx, wv);
          else {
#pragma unroll
            for (int i = 0; i < 8; ++i) wv[i] = 1.f;
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            o[i] = (dv[i] * wv[i] - c2 - (rv[i] - mu) * rs * c1) * rs;
            if (dr_out) o[i] += ev[i];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = (g[c][i] - c2 - xh[c][i] * c1) * rs;
          if (dr_out) {
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] += e[c][i];
          }
        }
        store8<T>(dr_in + base + idx, o);
        if (dh) {
          if (thr) {
            bool k[8];
            keep8(seed, offset, base + idx, thr, k);
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = k[i] ? o[i] * scale : 0.f;
          }
          store8<T>(dh + base + idx, o);
#pragma unroll
          for (int i = 0; i < 8; ++i) ah[c][i] += o[i];
        }
      }
    }
  }
  // reduce the 4 waves' partials through LDS, write one row of partials per workgroup
  float* parts[3] = {pw, pb, pbias};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (parts[a] == nullptr) continue;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < cols) {
        float* src = a == 0 ? aw[c] : (a == 1 ? ab[c] : ah[c]);
        store8<float>(red_lds + (size_t)wid * cols + idx, src);
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < cols; i += blockDim.x) {
      float t = red_lds[i] + red_lds[cols + i] + red_lds[2 * cols + i] + red_lds[3 * cols + i];
      parts[a][(size_t)blockIdx.x * cols + i] = t;
    }
  }
}

#define ADL_BWD_ARGS                                                                                         \
  const T* __restrict__ dy, const T* __restrict__ dr_out, const T* __restrict__ r, const W* __restrict__ w,  \
      const float* __restrict__ mean, const float* __restrict__ rstd, T* __restrict__ dr_in, T* __restrict__ dh, \
      float* __restrict__ pw, float* __restrict__ pb, float* __restrict__ pbias, int rows, int cols, uint32_t thr, \
      float scale, uint64_t seed, uint64_t offset, const uint64_t* __restrict__ dseq
template <typename T, typename W, int C>
__global__ void __launch_bounds__(256) adl_bwd_k(ADL_BWD_ARGS) {
  adl_bwd_body<T, W, C, false>(dy, dr_out, r, w, mean, rstd, dr_in, dh, pw, pb, pbias, rows, cols, thr, scale, seed,
                               offset, dseq);
}
template <typename T, typename W, int C>
__global__ void __launch_bounds__(256, 3) adl_bwd2_k(ADL_BWD_ARGS) {
  adl_bwd_body<T, W, C, true>(dy, dr_out, r, w, mean, rstd, dr_in, dh, pw, pb, pbias, rows, cols, thr, scale, seed,
                              offset, dseq);
}
#undef ADL_BWD_ARGS

// out[c] = sum_b part[b][c]; workgroup = 16 columns x 16 row slices
template <typename O>
__global__ void __launch_bounds__(256) colsum16_k(const float* __restrict__ part, O* __restrict__ out, int nblk,
                                                  int cols, int acc) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (c < cols)
    for (int b = rg; b < nblk; b += 16) s += part[(size_t)b * cols + c];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][cl];
    if (acc) t += Cvt<O>::to(out[c]);  // accumulate into an existing gradient
    out[c] = Cvt<O>::from(t);
  }
}

// out[c] (+)= sum_b part[b][c], cols % 4 == 0: a workgroup = 16 column quads (64 columns) x 16
// row slices; each lane keeps four 16-B loads in flight (the 16-column form issued one 4-B load
// at a time per lane and ran latency-bound at ~0.35 TB/s)
template <typename O>
__device__ __forceinline__ void colsum4_body(const float* __restrict__ part, O* __restrict__ out, int nblk, int cols,
                                             int acc) {
  __shared__ float4 red[16][17];
  const int cq = threadIdx.x & 15, rs = threadIdx.x >> 4;
  const int c = (blockIdx.x * 16 + cq) * 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < cols) {
    const float* p = part + c;
    int b = rs;
    for (; b + 48 < nblk; b += 64) {
      const float4 v0 = *reinterpret_cast<const float4*>(p + (size_t)b * cols);
      const float4 v1 = *reinterpret_cast<const float4*>(p + (size_t)(b + 16) * cols);
      const float4 v2 = *reinterpret_cast<const float4*>(p + (size_t)(b + 32) * cols);
      const float4 v3 = *reinterpret_cast<const float4*>(p + (size_t)(b + 48) * cols);
      a.x += (v0.x + v1.x) + (v2.x + v3.x);
      a.y += (v0.y + v1.y) + (v2.y + v3.y);
      a.z += (v0.z + v1.z) + (v2.z + v3.z);
      a.w += (v0.w + v1.w) + (v2.w + v3.w);
    }
    for (; b < nblk; b += 16) {
      const float4 v = *reinterpret_cast<const float4*>(p + (size_t)b * cols);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[rs][cq] = a;
  __syncthreads();
  if (rs == 0 && c < cols) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 16; ++i) { t.x += red[i][cq].x; t.y += red[i][cq].y; t.z += red[i][cq].z; t.w += red[i][cq].w; }
    const float r[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) out[c + e] = Cvt<O>::from(r[e] + (acc ? Cvt<O>::to(out[c + e]) : 0.f));
  }
}
template <typename O>
__global__ void __launch_bounds__(256) colsum4_k(const float* __restrict__ part, O* __restrict__ out, int nblk,
                                                 int cols, int acc) {
  colsum4_body<O>(part, out, nblk, cols, acc);
}
// up to 3 independent column reductions of one shape in ONE launch (grid.y = job): the LayerNorm
// weight / bias and the residual-branch bias gradients of one add+dropout+LN backward
struct ColsumJobs {
  const float* part[3];
  void* out[3];
  int acc[3];
};
template <typename O>
__global__ void __launch_bounds__(256) colsum4_multi_k(ColsumJobs jobs, int nblk, int cols) {
  const int j = blockIdx.y;
  colsum4_body<O>(jobs.part[j], static_cast<O*>(jobs.out[j]), nblk, cols, jobs.acc[j]);
}

}  // namespace pra

using namespace pra;

#define ADL_DISPATCH_C(cols, KER, ...)                      \
  do {                                                      \
    int _ch = ((cols) / 8 + 63) / 64;                       \
    if (_ch <= 1) KER(1, __VA_ARGS__);                      \
    else if (_ch <= 2) KER(2, __VA_ARGS__);                 \
    else if (_ch <= 4) KER(4, __VA_ARGS__);                 \
    else KER(8, __VA_ARGS__);                               \
  } while (0)

extern "C" {
int pra_adl_supported(int cols) { return (cols % 8 == 0 && cols <= 4096) ? 1 : 0; }

void pra_adl_fwd(const void* x, const void* h, const void* hbias, const void* w, const void* b, void* r_out,
                 void* y, float* mean, float* rstd, int rows, int cols, float eps, float p, uint64_t seed,
                 uint64_t offset, const uint64_t* dseq, int dt, int dtw, hipStream_t s) {
  if (!rows) return;
  uint32_t thr = (h && p > 0.f) ? (uint32_t)(p * 65536.f + 0.5f) : 0u;
  float scale = thr ? 1.f / (1.f - p) : 1.f;
  dim3 grid((rows + 3) / 4);
#define K_FWD(CC, TX, TW)                                                                                  \
  hipLaunchKernelGGL((adl_fwd_k<TX, TW, CC>), grid, dim3(256), 0, s, (const TX*)x, (const TX*)h,             \
                     (const TX*)hbias, (const TW*)w, (const TW*)b, (TX*)r_out, (TX*)y, mean, rstd, rows, cols, \
                     eps, thr, scale, seed, offset, dseq)
  PRA_DISPATCH_FLOAT(dt, TX, {
    if (dtw == dt) { ADL_DISPATCH_C(cols, K_FWD, TX, TX); }
    else { ADL_DISPATCH_C(cols, K_FWD, TX, float); }
  });
#undef K_FWD
}

void pra_adl_bwd(const void* dy, const void* dr_out, const void* r, const void* w, const float* mean,
                 const float* rstd, void* dr_in, void* dh, float* pw, float* pb, float* pbias, int rows, int cols,
                 int nblk, float p, uint64_t seed, uint64_t offset, const uint64_t* dseq, int dt, int dtw,
                 hipStream_t s) {
  if (!rows) return;
  uint32_t thr = (dh && p > 0.f) ? (uint32_t)(p * 65536.f + 0.5f) : 0u;
  float scale = thr ? 1.f / (1.f - p) : 1.f;
  size_t lds = (size_t)4 * cols * sizeof(float);
  static const bool two = !(getenv("PRA_ADL_BWD") && atoi(getenv("PRA_ADL_BWD")) == 1);
#define K_BWD(CC, TX, TW)                                                                                  \
  if (two)                                                                                                 \
    hipLaunchKernelGGL((adl_bwd2_k<TX, TW, CC>), dim3(nblk), dim3(256), lds, s, (const TX*)dy, (const TX*)dr_out, \
                       (const TX*)r, (const TW*)w, mean, rstd, (TX*)dr_in, (TX*)dh, pw, pb, pbias, rows, cols, thr, \
                       scale, seed, offset, dseq);                                                         \
  else                                                                                                     \
    hipLaunchKernelGGL((adl_bwd_k<TX, TW, CC>), dim3(nblk), dim3(256), lds, s, (const TX*)dy, (const TX*)dr_out, \
                       (const TX*)r, (const TW*)w, mean, rstd, (TX*)dr_in, (TX*)dh, pw, pb, pbias, rows, cols, thr, \
                       scale, seed, offset, dseq)
  PRA_DISPATCH_FLOAT(dt, TX, {
    if (dtw == dt) { ADL_DISPATCH_C(cols, K_BWD, TX, TX); }
    else { ADL_DISPATCH_C(cols, K_BWD, TX, float); }
  });
#undef K_BWD
}

// njobs <= 3 reductions part[j] [nblk][cols] -> out[j] (+= when acc[j]), one dtype; cols % 4 == 0
int pra_colsum_multi(const float* const* part, void* const* out, const int* acc, int njobs, int nblk, int cols,
                     int dto, hipStream_t s) {
  if (njobs < 1 || njobs > 3 || cols % 4) return -1;
  ColsumJobs jb{};
  for (int j = 0; j < njobs; ++j) {
    if (((uintptr_t)part[j] & 15) != 0) return -1;
    jb.part[j] = part[j];
    jb.out[j] = out[j];
    jb.acc[j] = acc[j];
  }
  PRA_DISPATCH_FLOAT(dto, TO, hipLaunchKernelGGL((colsum4_multi_k<TO>), dim3((cols + 63) / 64, njobs), dim3(256), 0,
                                                 s, jb, nblk, cols));
  return 0;
}
void pra_colsum16(const float* part, void* out, int nblk, int cols, int dto, int acc, hipStream_t s) {
  if (cols % 4 == 0 && ((uintptr_t)part & 15) == 0) {
    PRA_DISPATCH_FLOAT(dto, TO, hipLaunchKernelGGL((colsum4_k<TO>), dim3((cols + 63) / 64), dim3(256), 0, s,
                                                   part, (TO*)out, nblk, cols, acc));
    return;
  }
  PRA_DISPATCH_FLOAT(dto, TO, hipLaunchKernelGGL((colsum16_k<TO>), dim3((cols + 15) / 16), dim3(256), 0, s,
                                                 part, (TO*)out, nblk, cols, acc));
}
}
