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

template <typename T>
__global__ void __launch_bounds__(256) max_pool_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                      uint8_t* __restrict__ idx, PoolGeom g, int64_t nvec) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvec) return;
  const int CV = g.C >> 3;
  const int cv = (int)(v % CV);
  int64_t p = v / CV;
  const int wo = (int)(p % g.Wo); p /= g.Wo;
  const int ho = (int)(p % g.Ho);
  const int n = (int)(p / g.Ho);
  float m[8], t[8];
  uint32_t arg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { m[e] = -INFINITY; arg[e] = 0; }
  const int h0 = ho * g.SH - g.PH, w0 = wo * g.SW - g.PW;
  for (int kh = 0; kh < g.KH; ++kh) {
    const int h = h0 + kh;
    if ((unsigned)h >= (unsigned)g.H) continue;
    for (int kw = 0; kw < g.KW; ++kw) {
      const int w = w0 + kw;
      if ((unsigned)w >= (unsigned)g.W) continue;
      load8<T>(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + cv * 8, t);
      const uint32_t tap = kh * g.KW + kw;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (t[e] > m[e] || (t[e] != t[e] && m[e] == m[e])) { m[e] = t[e]; arg[e] = tap; }
    }
  }
  store8<T>(y + v * 8, m);
  uint2 packed;
  packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
  *reinterpret_cast<uint2*>(idx + v * 8) = packed;
}

template <typename T>
__global__ void __launch_bounds__(256) max_pool_bwd_k(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                      T* __restrict__ dx, PoolGeom g, int64_t nvec) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvec) return;
  const int CV = g.C >> 3;
  const int cv = (int)(v % CV);
  int64_t p = v / CV;
  const int w = (int)(p % g.W); p /= g.W;
  const int h = (int)(p % g.H);
  const int n = (int)(p / g.H);
  // output rows whose window [ho*SH-PH, ho*SH-PH+KH) contains h
  const int hh = h + g.PH, ww = w + g.PW;
  const int ho_lo = hh >= g.KH ? (hh - g.KH) / g.SH + 1 : 0, ho_hi = min(hh / g.SH, g.Ho - 1);
  const int wo_lo = ww >= g.KW ? (ww - g.KW) / g.SW + 1 : 0, wo_hi = min(ww / g.SW, g.Wo - 1);
  float acc[8], t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int ho = ho_lo; ho <= ho_hi; ++ho) {
    for (int wo = wo_lo; wo <= wo_hi; ++wo) {
      const uint32_t tap = (hh - ho * g.SH) * g.KW + (ww - wo * g.SW);
      const int64_t o = (((int64_t)n * g.Ho + ho) * g.Wo + wo) * g.C + cv * 8;
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
  store8<T>(dx + v * 8, acc);
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
  PRA_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL(pra::max_pool_fwd_k<T>, dim3(blocks), dim3(256), 0, s, (const T*)x, (T*)y, idx, g, nvec);
  });
  return 0;
}

extern "C" int pra_max_pool_bwd(const void* dy, const uint8_t* idx, void* dx, int N, int H, int W, int C, int Ho,
                                int Wo, int KH, int KW, int SH, int SW, int PH, int PW, int dt, hipStream_t s) {
  PoolGeom g{N, H, W, C, Ho, Wo, KH, KW, SH, SW, PH, PW};
  if (!pool_ok(g)) return -1;
  const int64_t nvec = (int64_t)N * H * W * (C / 8);
  const unsigned blocks = (unsigned)((nvec + 255) / 256);
  PRA_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL(pra::max_pool_bwd_k<T>, dim3(blocks), dim3(256), 0, s, (const T*)dy, idx, (T*)dx, g, nvec);
  });
  return 0;
}
