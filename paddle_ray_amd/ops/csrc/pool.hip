// Max pooling, channels-last (parity: paddle/phi/kernels/funcs/pooling.cu max pool forward /
// backward, e.g. ResNet's 3x3/s2 stem pool).
//   max_pool_fwd_k : one lane per (output pixel, 8 channels): scans the k x k window (taps outside
//                    the image skipped, first maximum wins as in the reference), writes y and the
//                    winning tap per channel as ONE BYTE (not an int64 index tensor).
//   max_pool_bwd_k : one lane per (input pixel, 8 channels): gathers dy from the <= ceil(k/s)^2
//                    windows that contain it whose stored tap is this pixel. No atomics, no
//                    zero-fill pass, dx written once with 16-B stores.
#include "common.h"

namespace pra {

struct PoolGeom {
  int N, H, W, C, Ho, Wo, KH, KW, SH, SW, PH, PW;
};

// I: the index type of the lane decomposition and the element offsets (uint32_t whenever the
// tensors have < 2^32 elements, int64_t otherwise).
// KC > 0: a KC x KC window known at compile time (ResNet's 3x3 stem pool): all KC^2 taps are
// loaded from clamped (always valid) addresses before the first compare, so the loads overlap
// instead of one dependent round trip per tap; out-of-image taps are masked in the compare.
template <typename T, typename I, int KC>
__global__ void __launch_bounds__(256) max_pool_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                      uint8_t* __restrict__ idx, PoolGeom g, I nvec) {
  const I v = (I)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvec) return;
  const I CV = g.C >> 3;
  const int cv = (int)(v % CV);
  I p = v / CV;
  const int wo = (int)(p % (I)g.Wo); p /= (I)g.Wo;
  const int ho = (int)(p % (I)g.Ho);
  const int n = (int)(p / (I)g.Ho);
  float m[8], t[8];
  uint32_t arg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { m[e] = -INFINITY; arg[e] = 0; }
  const int h0 = ho * g.SH - g.PH, w0 = wo * g.SW - g.PW;
  const T* xn = x + (I)n * g.H * g.W * g.C + cv * 8;
  if constexpr (KC > 0) {
    float tt[KC * KC][8];
#pragma unroll
    for (int kh = 0; kh < KC; ++kh)
#pragma unroll
      for (int kw = 0; kw < KC; ++kw) {
        const int h = min(max(h0 + kh, 0), g.H - 1), w = min(max(w0 + kw, 0), g.W - 1);
        load8<T>(xn + ((I)h * g.W + w) * g.C, tt[kh * KC + kw]);
      }
#pragma unroll
    for (int kh = 0; kh < KC; ++kh)
#pragma unroll
      for (int kw = 0; kw < KC; ++kw) {
        const bool in = (unsigned)(h0 + kh) < (unsigned)g.H && (unsigned)(w0 + kw) < (unsigned)g.W;
        const float* u = tt[kh * KC + kw];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (in && (u[e] > m[e] || (u[e] != u[e] && m[e] == m[e]))) { m[e] = u[e]; arg[e] = kh * KC + kw; }
      }
  } else {
    for (int kh = 0; kh < g.KH; ++kh) {
      const int h = h0 + kh;
      if ((unsigned)h >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int w = w0 + kw;
        if ((unsigned)w >= (unsigned)g.W) continue;
        load8<T>(xn + ((I)h * g.W + w) * g.C, t);
        const uint32_t tap = kh * g.KW + kw;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (t[e] > m[e] || (t[e] != t[e] && m[e] == m[e])) { m[e] = t[e]; arg[e] = tap; }
      }
    }
  }
  store8<T>(y + v * 8, m);
  uint2 packed;
  packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
  *reinterpret_cast<uint2*>(idx + v * 8) = packed;
}

// MW > 0: at most MW windows per dimension contain an input pixel (ceil(K/S) <= MW: 2 for the
// 3x3 / s2 stem pool); the MW^2 tap-index and dy loads are issued together from clamped
// addresses, then matched.
template <typename T, typename I, int MW>
__global__ void __launch_bounds__(256) max_pool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                      T* __restrict__ dx, PoolGeom g, I nvec) {
  const I v = (I)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvec) return;
  const I CV = g.C >> 3;
  const int cv = (int)(v % CV);
  I p = v / CV;
  const int w = (int)(p % (I)g.W); p /= (I)g.W;
  const int h = (int)(p % (I)g.H);
  const int n = (int)(p / (I)g.H);
  // output rows whose window [ho*SH-PH, ho*SH-PH+KH) contains h
  const int hh = h + g.PH, ww = w + g.PW;
  const int ho_lo = hh >= g.KH ? (hh - g.KH) / g.SH + 1 : 0, ho_hi = min(hh / g.SH, g.Ho - 1);
  const int wo_lo = ww >= g.KW ? (ww - g.KW) / g.SW + 1 : 0, wo_hi = min(ww / g.SW, g.Wo - 1);
  const I nbase = (I)n * g.Ho * g.Wo * g.C + cv * 8;
  float acc[8], t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  if constexpr (MW > 0) {
    float tt[MW * MW][8];
    uint2 pk[MW * MW];
#pragma unroll
    for (int i = 0; i < MW; ++i)
#pragma unroll
      for (int j = 0; j < MW; ++j) {
        const int ho = min(ho_lo + i, g.Ho - 1), wo = min(wo_lo + j, g.Wo - 1);
        const I o = nbase + ((I)ho * g.Wo + wo) * g.C;
        pk[i * MW + j] = *reinterpret_cast<const uint2*>(idx + o);
        load8<T>(dy + o, tt[i * MW + j]);
      }
#pragma unroll
    for (int i = 0; i < MW; ++i)
#pragma unroll
      for (int j = 0; j < MW; ++j) {
        const int ho = ho_lo + i, wo = wo_lo + j;
        const bool in = ho <= ho_hi && wo <= wo_hi;
        const uint32_t tap = (hh - ho * g.SH) * g.KW + (ww - wo * g.SW);
        const uint32_t a[2] = {pk[i * MW + j].x, pk[i * MW + j].y};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (in && ((a[e >> 2] >> (8 * (e & 3))) & 0xffu) == tap) acc[e] += tt[i * MW + j][e];
      }
  } else {
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const uint32_t tap = (hh - ho * g.SH) * g.KW + (ww - wo * g.SW);
        const I o = nbase + ((I)ho * g.Wo + wo) * g.C;
        const uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
        const uint32_t a[2] = {pk.x, pk.y};
        bool any = false;
#pragma unroll
        for (int e = 0; e < 8; ++e) any |= ((a[e >> 2] >> (8 * (e & 3))) & 0xffu) == tap;
        if (!any) continue;
        load8<T>(dy + o, t);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (((a[e >> 2] >> (8 * (e & 3))) & 0xffu) == tap) acc[e] += t[e];
      }
    }
  }
  store8<T>(dx + v * 8, acc);
}

// Filter of a KxK convolution's input gradient (stride 1): dst[c][ky][kx][o] =
// src[o][c][KH-1-ky][KW-1-kx] (OIHW -> flipped IHWO) in ONE pass, one lane per destination element
// (the torch flip + permute copy was two launches per 3x3 layer per step).
template <typename T>
__global__ void __launch_bounds__(256) wflip_t_k(const T* __restrict__ src, T* __restrict__ dst, int O, int C, int KH,
                                                 int KW, uint32_t n) {
  const uint32_t v = blockIdx.x * 256u + threadIdx.x;
  if (v >= n) return;
  const uint32_t o = v % (uint32_t)O;
  uint32_t r = v / (uint32_t)O;
  const uint32_t kx = r % (uint32_t)KW;
  r /= (uint32_t)KW;
  const uint32_t ky = r % (uint32_t)KH;
  const uint32_t c = r / (uint32_t)KH;
  dst[v] = src[((o * C + c) * KH + (KH - 1 - ky)) * KW + (KW - 1 - kx)];
}

// 2x2 space-to-depth with zero padding, channels-last: x [N][H][W][C] ->
// y [N][(H+2P)/2][(W+2P)/2][CO], y[n][i][j][(2dy+dx)*C + c] = x[n][2i+dy-P][2j+dx-P][c] (zero
// outside the image and in the channels 4C..CO-1). Feeds the stride-2 stem convolution as a
// stride-1 one on the 16-channel image (gemm_lds.hip pixel-pitch mode). One lane per output
// pixel, 16-B stores.
template <typename T>
__global__ void __launch_bounds__(256) s2d2_k(const T* __restrict__ x, T* __restrict__ y, int H, int W, int C, int P,
                                              int Hs, int Ws, int CO, int64_t npix) {
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= npix) return;
  const int j = (int)(pix % Ws);
  const int64_t t = pix / Ws;
  const int i = (int)(t % Hs);
  const int64_t n = t / Hs;
  for (int q = 0; q < CO / 8; ++q) {
    uint32_t w4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint16_t h2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = q * 8 + 2 * e + u, blk = k / C, c = k - blk * C;
        const int hh = 2 * i + (blk >> 1) - P, ww = 2 * j + (blk & 1) - P;
        h2[u] = 0;
        if (blk < 4 && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W)
          h2[u] = reinterpret_cast<const uint16_t*>(x)[((n * H + hh) * W + ww) * C + c];
      }
      w4[e] = (uint32_t)h2[0] | ((uint32_t)h2[1] << 16);
    }
    *reinterpret_cast<uint4*>(y + pix * CO + q * 8) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}

}  // namespace pra

extern "C" int pra_space_to_depth2(const void* x, void* y, int N, int H, int W, int C, int P, int CO, int dt,
                                   hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || P < 0 || CO % 8 || CO < 4 * C || (H + 2 * P) % 2 || (W + 2 * P) % 2)
    return -1;
  if (dt != pra::kBF16 && dt != pra::kF16) return -1;
  const int Hs = (H + 2 * P) / 2, Ws = (W + 2 * P) / 2;
  const int64_t npix = (int64_t)N * Hs * Ws;
  pra::s2d2_k<uint16_t><<<(unsigned)((npix + 255) / 256), 256, 0, s>>>(
      static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), H, W, C, P, Hs, Ws, CO, npix);
  return 0;
}

namespace pra {
// Global average pooling backward, channels-last: dx[n][p][c] = dy[n][c] * scale for all HW
// pixels p (a broadcast write; torch's expand + copy runs a non-vectorised strided kernel)
template <typename T>
__global__ void __launch_bounds__(256) gap_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int HW, int CV,
                                                 float scale, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * 256) {
    const int cv = (int)(v % CV);
    const int64_t n = v / ((int64_t)HW * CV);
    float g[8];
    load8<T>(dy + (n * CV + cv) * 8, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= scale;
    store8<T>(dx + v * 8, g);
  }
}
}  // namespace pra

extern "C" int pra_gap_bwd(const void* dy, void* dx, int N, int HW, int C, int dt, hipStream_t s) {
  if (N <= 0 || HW <= 0 || C % 8) return -1;
  const int64_t nvec = (int64_t)N * HW * (C / 8);
  const int64_t want = (nvec + 255) / 256;
  const unsigned blocks = (unsigned)(want < 4096 ? want : 4096);
  const float scale = 1.f / (float)HW;
  PRA_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL(pra::gap_bwd_k<T>, dim3(blocks), dim3(256), 0, s, (const T*)dy, (T*)dx, HW, C / 8, scale, nvec);
  });
  return 0;
}

using pra::PoolGeom;

static bool pool_ok(const PoolGeom& g) {
  return g.C % 8 == 0 && g.KH > 0 && g.KW > 0 && g.KH * g.KW <= 255 && g.SH > 0 && g.SW > 0 && g.PH >= 0 &&
         g.PW >= 0 && g.PH < g.KH && g.PW < g.KW && g.Ho > 0 && g.Wo > 0;
}

// x [N][H][W][C] -> y [N][Ho][Wo][C], idx [N][Ho][Wo][C] uint8 (winning tap kh*KW+kw)
extern "C" int pra_max_pool_fwd(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                                int KH, int KW, int SH, int SW, int PH, int PW, int dt, hipStream_t s) {
  PoolGeom g{N, H, W, C, Ho, Wo, KH, KW, SH, SW, PH, PW};
  if (!pool_ok(g)) return -1;
  const int64_t nvec = (int64_t)N * Ho * Wo * (C / 8);
  const unsigned blocks = (unsigned)((nvec + 255) / 256);
  const bool narrow = nvec * 8 < ((int64_t)1 << 32) && (int64_t)N * H * W * C < ((int64_t)1 << 32);
  PRA_DISPATCH_FLOAT(dt, T, {
    if (narrow && KH == 3 && KW == 3)
      hipLaunchKernelGGL((pra::max_pool_fwd_k<T, uint32_t, 3>), dim3(blocks), dim3(256), 0, s, (const T*)x, (T*)y, idx,
                         g, (uint32_t)nvec);
    else if (narrow)
      hipLaunchKernelGGL((pra::max_pool_fwd_k<T, uint32_t, 0>), dim3(blocks), dim3(256), 0, s, (const T*)x, (T*)y, idx,
                         g, (uint32_t)nvec);
    else
      hipLaunchKernelGGL((pra::max_pool_fwd_k<T, int64_t, 0>), dim3(blocks), dim3(256), 0, s, (const T*)x, (T*)y, idx,
                         g, nvec);
  });
  return 0;
}

extern "C" int pra_max_pool_bwd(const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C, int Ho,
                                int Wo, int KH, int KW, int SH, int SW, int PH, int PW, int dt, hipStream_t s) {
  PoolGeom g{N, H, W, C, Ho, Wo, KH, KW, SH, SW, PH, PW};
  if (!pool_ok(g)) return -1;
  const int64_t nvec = (int64_t)N * H * W * (C / 8);
  const unsigned blocks = (unsigned)((nvec + 255) / 256);
  const bool narrow = nvec * 8 < ((int64_t)1 << 32) && (int64_t)N * Ho * Wo * C < ((int64_t)1 << 32);
  PRA_DISPATCH_FLOAT(dt, T, {
    if (narrow && (KH + SH - 1) / SH <= 2 && (KW + SW - 1) / SW <= 2)
      hipLaunchKernelGGL((pra::max_pool_bwd_k<T, uint32_t, 2>), dim3(blocks), dim3(256), 0, s, (const T*)dy, idx,
                         (T*)dx, g, (uint32_t)nvec);
    else if (narrow)
      hipLaunchKernelGGL((pra::max_pool_bwd_k<T, uint32_t, 0>), dim3(blocks), dim3(256), 0, s, (const T*)dy, idx,
                         (T*)dx, g, (uint32_t)nvec);
    else
      hipLaunchKernelGGL((pra::max_pool_bwd_k<T, int64_t, 0>), dim3(blocks), dim3(256), 0, s, (const T*)dy, idx,
                         (T*)dx, g, nvec);
  });
  return 0;
}

extern "C" int pra_wflip_t(const void* src, void* dst, int O, int C, int KH, int KW, int dt, hipStream_t s) {
  const int64_t n = (int64_t)O * C * KH * KW;
  if (O <= 0 || C <= 0 || KH <= 0 || KW <= 0 || n >= ((int64_t)1 << 32)) return -1;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  PRA_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL(pra::wflip_t_k<T>, dim3(blocks), dim3(256), 0, s, (const T*)src, (T*)dst, O, C, KH, KW,
                       (uint32_t)n);
  });
  return 0;
}
