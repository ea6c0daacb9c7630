// Device side of the LDS-DMA MFMA GEMM (the kernel template, its operand stagers and the
// split-K / column-sum reductions), shared by the translation units that instantiate it:
// gemm_lds.hip (8-wave configurations, convolutions, the C entry points) and gemm_w4.hip
// (the 4-wave 128x128-per-wave configuration). Design notes: gemm_lds.hip.
#pragma once
#include "common.h"
#include <stdlib.h>
#include <type_traits>

namespace pra {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
template <typename T> struct V8;
template <> struct V8<bf16> { typedef __bf16 type __attribute__((ext_vector_type(8))); };
template <> struct V8<f16> { typedef _Float16 type __attribute__((ext_vector_type(8))); };

template <typename T>
__device__ __forceinline__ f32x4 mma(typename V8<T>::type a, typename V8<T>::type b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mma<bf16>(V8<bf16>::type a, V8<bf16>::type b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mma<f16>(V8<f16>::type a, V8<f16>::type b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// One wave per SIMD (W4: 128x128 outputs per wave) holds 256 fp32 accumulators: the MFMA is
// issued from inline asm with the accumulator constrained to AGPRs and the operands to VGPRs.
// With the builtin, the register allocator spreads the accumulators over both files and
// shuffles them with v_accvgpr_read/write/mov inside the K loop (or, before the lambdas below
// were force-inlined, spilled them to scratch). The asm is opaque to the hazard recognizer:
// the kernel pads the AGPR-write -> v_accvgpr_read hazard itself before its epilogue.
template <typename T>
__device__ __forceinline__ void mma_agpr(typename V8<T>::type a, typename V8<T>::type b, f32x4& c);
template <>
__device__ __forceinline__ void mma_agpr<bf16>(V8<bf16>::type a, V8<bf16>::type b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
template <>
__device__ __forceinline__ void mma_agpr<f16>(V8<f16>::type a, V8<f16>::type b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <typename T> __device__ __forceinline__ float to_f(uint16_t u);
template <> __device__ __forceinline__ float to_f<bf16>(uint16_t u) { return bf2f(u); }
template <> __device__ __forceinline__ float to_f<f16>(uint16_t u) { return (float)__builtin_bit_cast(_Float16, u); }
template <typename T> __device__ __forceinline__ uint32_t pack2(float a, float b);
template <> __device__ __forceinline__ uint32_t pack2<bf16>(float a, float b) { return pack_bf2(a, b); }
template <> __device__ __forceinline__ uint32_t pack2<f16>(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)b) << 16);
}

// kGelu*D: forward GELU whose Z output receives gelu'(pre-activation) instead of the pre-activation
// (the only thing the backward needs from it); kMulZ: C = acc * Z, the backward's dGELU as one
// multiply (with the derivative saved by the forward, the dgrad epilogue carries no transcendental
// work: profiles/r4/fused_dgelu_epilogue.md measured that VALU serialised behind the K loop).
enum Epi : int {
  kNone = 0, kGeluErf = 1, kGeluTanh = 2, kRelu = 3, kDGeluErf = 4, kDGeluTanh = 5,
  kGeluErfD = 6, kGeluTanhD = 7, kMulZ = 8, kBnG = 9
};
// kBnG (implicit-GEMM conv dgrad feeding a BatchNorm+ReLU backward): C = acc masked by the ReLU
// keep-bits (mbits, 1 bit per element), colsum = sum of that g, colsq = sum of g * (Z - cshift)
// with Z the BN input and cshift its batch mean -- the BN backward's two reductions.
// epilogues that read Z and scale the product by a per-element factor (the dgrad side)
constexpr bool epi_scales(int E) { return E == kDGeluErf || E == kDGeluTanh || E == kMulZ; }
// forward GELUs that store the derivative into Z
constexpr bool epi_gd(int E) { return E == kGeluErfD || E == kGeluTanhD; }

// tanh-GELU in sigmoid form: 0.5 (1 + tanh(u)) = sigmoid(2u) with 2u = x (k1 + k3 x^2), so
//   gelu(x) = x s,   gelu'(x) = s + x s (1 - s) (k1 + 3 k3 x^2),   s = 1 / (1 + 2^(-2u log2 e))
// one v_exp + one v_rcp and ~9 FMA-class ops for BOTH values (the tanh form took ~19: the
// derivative-saving forward epilogue runs serialised behind the K loop at one wave per SIMD,
// profiles/r5/gemm_fwd_probe.log). Saturates cleanly: x -> -inf gives s = 0, x -> +inf s = 1.
constexpr float kGT1 = 1.5957691216057308f;   // 2 sqrt(2 / pi)
constexpr float kGT3 = 0.0713548162726009f;   // kGT1 * 0.044715
constexpr float kLog2e = 1.4426950408889634f;
__device__ __forceinline__ float gelu_tanh_sig(float x, float x2) {
  const float e = __builtin_amdgcn_exp2f(-x * fmaf(kGT3 * kLog2e, x2, kGT1 * kLog2e));
  return __builtin_amdgcn_rcpf(1.f + e);
}
__device__ __forceinline__ float gelu_tanh(float x) { return x * gelu_tanh_sig(x, x * x); }
__device__ __forceinline__ float dgelu_tanh(float x) {
  const float x2 = x * x, s = gelu_tanh_sig(x, x2);
  return fmaf(x * s * (1.f - s), fmaf(3.f * kGT3, x2, kGT1), s);
}
__device__ __forceinline__ float gelu_erf(float x) { return gelu_erf_fast(x); }
__device__ __forceinline__ float dgelu_erf(float x) { return dgelu_erf_fast(x); }

template <int E>
__device__ __forceinline__ float act(float x) {
  if (E == kGeluErf || E == kGeluErfD) return gelu_erf(x);
  if (E == kGeluTanh || E == kGeluTanhD) return gelu_tanh(x);
  if (E == kRelu) return fmaxf(x, 0.f);
  return x;
}
// tanh-GELU and its derivative for two elements as packed f32 math (v_pk_mul / v_pk_fma / v_pk_add:
// two lanes' worth per instruction in the serialised GEMM epilogue; the exp / rcp stay scalar)
typedef float pf32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf32x2 gelu_tanh_d2(pf32x2 x, pf32x2& d) {
  const pf32x2 x2 = x * x;
  const pf32x2 u = -x * (x2 * (kGT3 * kLog2e) + (kGT1 * kLog2e));
  pf32x2 e;
  e.x = __builtin_amdgcn_exp2f(u.x);
  e.y = __builtin_amdgcn_exp2f(u.y);
  const pf32x2 den = e + 1.f;
  pf32x2 sg;
  sg.x = __builtin_amdgcn_rcpf(den.x);
  sg.y = __builtin_amdgcn_rcpf(den.y);
  const pf32x2 y = x * sg;
  d = (y * (1.f - sg)) * (x2 * (3.f * kGT3) + kGT1) + sg;
  return y;
}

// erf-GELU and its derivative for two elements, packed f32 (erf_from_exp's rational
// approximation; exp / rcp / sign transfer per element)
__device__ __forceinline__ pf32x2 gelu_erf_d2(pf32x2 x, pf32x2& d) {
  const pf32x2 u = x * 0.70710678118654752f;
  const pf32x2 w = -(u * u) * kLog2e;
  pf32x2 e, t;
  e.x = __builtin_amdgcn_exp2f(w.x);
  e.y = __builtin_amdgcn_exp2f(w.y);
  const pf32x2 den = pf32x2{fabsf(u.x), fabsf(u.y)} * 0.3275911f + 1.f;
  t.x = __builtin_amdgcn_rcpf(den.x);
  t.y = __builtin_amdgcn_rcpf(den.y);
  const pf32x2 p =
      t * (t * (t * (t * (t * 1.061405429f + -1.453152027f) + 1.421413741f) + -0.284496736f) + 0.254829592f);
  const pf32x2 m = 1.f - p * e;  // erf(|u|)
  const pf32x2 er = pf32x2{copysignf(m.x, u.x), copysignf(m.y, u.y)};
  const pf32x2 h = er * 0.5f + 0.5f;
  d = (x * 0.3989422804014327f) * e + h;
  return x * h;
}

// gelu(x) and gelu'(x) sharing the one transcendental
template <int E>
__device__ __forceinline__ float act_d(float x, float& d) {
  if constexpr (E == kGeluTanhD) {
    const float x2 = x * x, sg = gelu_tanh_sig(x, x2), y = x * sg;
    d = fmaf(y * (1.f - sg), fmaf(3.f * kGT3, x2, kGT1), sg);
    return y;
  } else {
    const float u = x * 0.70710678118654752f;
    const float e = __expf(-u * u);
    const float h = 0.5f * (1.f + erf_from_exp(u, e));
    d = h + x * 0.3989422804014327f * e;
    return x * h;
  }
}
// the dgrad-side factor of Z
template <int E>
__device__ __forceinline__ float zfac(float z) {
  if constexpr (E == kMulZ) return z;
  else if constexpr (E == kDGeluErf) return dgelu_erf(z);
  else return dgelu_tanh(z);
}

constexpr int BM = 256, BN = 256, BKT = 64;  // the GEMM tile (conv configs below narrow BN)

// Lanes per output quad of splitk_reduce_k: enough to fill the chip when the output is small and
// the split count large.
inline int splitk_groups(int64_t quads, int splits) {
  static const int gmax = getenv("PRA_SPLITK_GMAX") ? atoi(getenv("PRA_SPLITK_GMAX")) : 64;   // A/B knob
  int G = 1;
  while (2 * G <= gmax && 2 * G <= splits && quads * G < 262144) G *= 2;
  return G;
}

// Phase stamps for diagnostic builds only (gemm_probe.hip defines PRA_GEMM_STAMPS 1; the
// library's kernels compile them out): lane 0 of wave 0 of each workgroup writes 8 words into
// the (otherwise unused) ws buffer of a non-split launch: shader clock at entry / loop start /
// loop end / exit, the 100 MHz real-time clock at entry / exit, HW_ID and XCC_ID.
#ifndef PRA_GEMM_STAMPS
#define PRA_GEMM_STAMPS 0
#endif
#define PRA_STAMP(k, v)                                                                            \
  do {                                                                                             \
    if constexpr (PRA_GEMM_STAMPS) {                                                               \
      if (threadIdx.x == 0)                                                                        \
        reinterpret_cast<volatile unsigned long long*>(ws)[(size_t)blockIdx.x * 16 + (k)] = (v);  \
    }                                                                                              \
  } while (0)
// in-loop section clocks (default K-step body): PRA_TMARK(i) takes shader clock mark i of the
// K-step, PRA_TACC adds the three section lengths to per-thread sums stored at words 8..10
#define PRA_TMARK(i)                                                                               \
  do {                                                                                             \
    if constexpr (PRA_GEMM_STAMPS) pra_tm[i] = __builtin_amdgcn_s_memtime();                      \
  } while (0)
#define PRA_TACC()                                                                                 \
  do {                                                                                             \
    if constexpr (PRA_GEMM_STAMPS) {                                                               \
      pra_ts[0] += pra_tm[1] - pra_tm[0];                                                          \
      pra_ts[1] += pra_tm[2] - pra_tm[1];                                                          \
      pra_ts[2] += pra_tm[3] - pra_tm[2];                                                          \
    }                                                                                              \
  } while (0)

// Wave layouts of a BM_ x BN_ tile: WR x WC waves, each (BM_/WR) x (BN_/WC) outputs.
//   W8: 256x256, 2 x 4 waves (128x64 each, 2 waves/SIMD, 32 accumulators)
//   W4: 256x256, 2 x 2 waves (128x128 each, 1 wave/SIMD, 64 accumulators in AGPRs)
//   C128 / C64: narrow-N tiles for convolutions with 128 / 64 output channels (256x128 and
//       512x64, 64x64 per wave): a 256-wide tile would leave half / three quarters of its
//       MFMAs on padding columns. Their B operand must be K-contiguous (BK = true).
// Each K-step stages A [BM][64] and B [BN][64] (or [64][BN]) images, double-buffered.
//   ILV: one non-MFMA instruction (an LDS-DMA issue or a fragment read) after each MFMA of a
//       segment instead of a burst between MFMA groups (one wave per SIMD has no partner wave
//       to cover a burst)
//   BUF: operand DMA as MUBUF buffer_load ... lds instead of global_load_lds
//   PIPE: two barriers per K-step and the refill DMA issued in half 0 (see kstep_p): every DMA
//       has at least two k-halves of lead instead of one
//   TS: the two-barrier "read early, refill early, wait late" schedule (see kstep_t): each K-step's
//       second-half fragments are read in the first MFMAs of its first half, so a barrier two
//       thirds into that half frees the slot for the K-step+2 refill; the next K-step's first
//       fragments are read only in the last MFMAs of the second half, after a counted vmcnt that
//       leaves the refill in flight -> every DMA piece has ~1.5 K-steps of lead (the loop shape
//       of the 256x256x64 MFMA16 kernels hipBLASLt ships for gfx950, measured 84 % MFMA-busy)
//   SC1: operand DMA with the sc1 cache policy (bypass the CU's vector L1: LDS-DMA data never
//       benefits from L1, and the loads then do not evict / thrash it)
template <int WR_, int WC_, int BM_ = 256, int BN_ = 256, bool ILV_ = false, bool BUF_ = false,
          bool PIPE_ = false, bool TS_ = false, bool SC1_ = false>
struct WCfg {
  static constexpr int WR = WR_, WC = WC_, NT = 64 * WR_ * WC_, BM = BM_, BN = BN_;
  static constexpr bool ILV = ILV_, BUF = BUF_, PIPE = PIPE_, TS = TS_, SC1 = SC1_;
  static constexpr int TI = BM_ / WR_ / 16, TJ = BN_ / WC_ / 16;  // 16x16 MFMA tiles per wave
  static constexpr int IMGA = BM_ * BKT * 2, IMGB = BN_ * BKT * 2, SLOT = IMGA + IMGB;
  static constexpr int NDA = IMGA / (NT * 16), NDB = IMGB / (NT * 16);  // glds per thread per K-step
  static constexpr int EPI = 128 * (BN_ + 4) * 4;  // epilogue image: 128 rows of fp32, padded pitch
  static constexpr int LDS = 2 * SLOT > EPI ? 2 * SLOT : EPI;
};
using W8 = WCfg<2, 4>;
using W4 = WCfg<2, 2, 256, 256, true>;  // instantiated in gemm_w4.hip
using C128 = WCfg<4, 2, 256, 128>;
using C64 = WCfg<8, 1, 512, 64>;

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt left unconstrained)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// MC image [64 k][256] (512-B rows): 16-B chunk ^= mc_swz(k) makes the two ds_read_b64_tr_b16
// of a 32-lane half (k rows 8g+q, g = 0,1, q = 0..3) hit 16 distinct slots of the bank row.
__device__ __forceinline__ int mc_swz(int k) { return 2 * ((k & 3) | ((k >> 1) & 4)); }
// KC image [256 rows][64 k] (128-B rows): 16-B chunk ^= (row>>1)&7. ds_read_b128 serves lanes in
// the groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32); with this XOR each group's 16 lanes hit
// 16 distinct 16-B slots (conflict-free).
__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 7; }

// Per-thread DMA plan for one operand image (NDMA glds per thread per K-step). A K-step moves
// whole 128-B lines of every row (BK = 64 bf16), so each L2 line is requested once.
// KC image: position P (16-B chunk 0..2047) = row P>>3, slot P&7 holds global chunk (P&7)^kc_swz(row).
// MC image (MCW columns: 256, or 128 for narrow tiles): position P = k-row P/(MCW/8), slot
// P%(MCW/8) holds global chunk (P%(MCW/8))^mc_swz(k) (mc_swz < 16 keeps it inside a 128-wide row).
template <bool KC, int NT, int NDMA, bool BUF = false, int MCW = 256, bool SC1 = false>
struct Dma {
  static constexpr int MCC = MCW / 8;  // 16-B chunks per k-row of the MC image
  uint32_t voff[NDMA];  // per-lane byte offsets of the chunks this thread stages
  uint64_t base;        // wave-uniform operand base (SGPRs); advanced per K-step
  uint64_t step;        // bytes per K-step
  __device__ __forceinline__ void init(const uint16_t* b, int ld, int r0, int rmax, int tid) {
#pragma unroll
    for (int n = 0; n < NDMA; ++n) {
      const int P = n * NT + tid;
      if (KC) {
        const int row = P >> 3, c = (P & 7) ^ kc_swz(row);
        const int r = min(r0 + row, rmax);
        voff[n] = (uint32_t)(((int64_t)r * ld + 8 * c) * 2);
      } else {
        const int k = P / MCC, c = (P % MCC) ^ mc_swz(k);
        const int col = min(r0 + 8 * c, rmax);  // rmax = last valid 8-aligned chunk start
        voff[n] = (uint32_t)(((int64_t)k * ld + col) * 2);
      }
    }
    base = (uint64_t)b;
    step = KC ? (uint64_t)BKT * 2 : (uint64_t)BKT * ld * 2;
  }
  __device__ __forceinline__ void advance(int ksteps) { base += (uint64_t)ksteps * step; }
  __device__ __forceinline__ void issue1(uint32_t lds_img, int wave, int kt, int n) {
    const uint64_t g = base + (uint64_t)kt * step;
    // readfirstlane returns int: go through uint32_t so the low word is ZERO-extended
    const uint32_t glo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)g);
    const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(g >> 32));
    // wave-uniform LDS base in M0; the hardware adds lane*16. Issued from inline asm so the
    // compiler's waitcnt model does not see an LDS write in flight and never drains it with
    // vmcnt(0) ahead of the fragment reads: the explicit vmcnt in the K loop is the only wait.
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_img + (n * NT + wave * 64) * 16);
    if constexpr (BUF && SC1) {
      const u32x4 rs = {glo, ghi & 0xffffu, 0xffffffffu, 0x00020000u};
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen sc1 lds" ::"v"(voff[n]),
                   "s"(rs), "s"(dst)
                   : "memory");
    } else if constexpr (BUF) {
      // MUBUF form (raw buffer, stride 0, no range limit: the offsets are clamped in-bounds)
      const u32x4 rs = {glo, ghi & 0xffffu, 0xffffffffu, 0x00020000u};
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff[n]), "s"(rs),
                   "s"(dst)
                   : "memory");
    } else if constexpr (SC1) {
      const uint64_t gs = ((uint64_t)ghi << 32) | (uint64_t)glo;
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 sc1" ::"v"(voff[n]), "s"(gs),
                   "s"(dst)
                   : "memory");
    } else {
      const uint64_t gs = ((uint64_t)ghi << 32) | (uint64_t)glo;
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff[n]), "s"(gs), "s"(dst)
                   : "memory");
    }
  }
};

// Implicit-GEMM convolution operand A = im2col(x) for a channels-last input x [N][H][W][C]:
// row m = output pixel (n, ho, wo), column k = (kh, kw, c). With C % 64 == 0 a K-step (64 k)
// lies inside one filter tap, so every staged row segment is 128 contiguous bytes of one input
// pixel: the LDS-DMA gathers rows straight from x (per-lane source offsets), nothing is
// materialised. The zero padding is the buffer descriptor's range check: a tap that falls
// outside the image gets an offset past num_records and the DMA writes zeros to LDS.
// PP: the input's pixel pitch in elements (its stored channel count). PP == C for a plain
// convolution; PP < C lets a K-step of C = 64 columns span 64 / PP adjacent pixels of a
// narrow-channel input (the space-to-depth stem: a 4-wide tap row of 16-channel pixels is one
// contiguous 128-B segment), with taps counted in units of C columns.
struct ConvGeom {
  int Ho, Wo, H, W, C, KW, S, P, PP;
  // OS > 0 (sub-pixel phase of a stride-OS transposed convolution, the strided dgrad): output
  // row m = (n, i, j) of the Ho x Wo phase grid is written to pixel (n, OS*i, OS*j) of an
  // (OS*Ho) x (OS*Wo) image (the phase offset is folded into the output pointer)
  int OS = 0;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NT, int NDMA>
struct ConvDmaA {
  int pix[NDMA];       // element offset of x[n][ho*S-P][wo*S-P][8c] (may be negative) per staged chunk
  uint32_t hw[NDMA];   // (ho*S-P) << 16 | (wo*S-P) & 0xffff
  u32x4 rs;            // buffer descriptor of x (wave-uniform, SGPRs)
  int kt0;
  ConvGeom g;
  __device__ __forceinline__ void init(const uint16_t* x, const ConvGeom& cg, int m0, int M, int tid) {
    g = cg;
#pragma unroll
    for (int n = 0; n < NDMA; ++n) {
      const int P = n * NT + tid;
      const int row = P >> 3, c = (P & 7) ^ kc_swz(row);
      const int m = min(m0 + row, M - 1);
      const int wo = m % g.Wo, t = m / g.Wo, ho = t % g.Ho, img = t / g.Ho;
      const int hi = ho * g.S - g.P, wi = wo * g.S - g.P;
      pix[n] = ((img * g.H + hi) * g.W + wi) * g.PP + 8 * c;
      hw[n] = ((uint32_t)hi << 16) | ((uint32_t)wi & 0xffffu);
    }
    const uint64_t b = (uint64_t)x;
    rs[0] = __builtin_amdgcn_readfirstlane((uint32_t)b);
    rs[1] = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xffffu;  // stride 0
    rs[2] = __builtin_amdgcn_readfirstlane((uint32_t)((int64_t)M / (g.Ho * g.Wo) * g.H * g.W * g.PP * 2));
    rs[3] = 0x00020000u;
    kt0 = 0;
  }
  __device__ __forceinline__ void advance(int ksteps) { kt0 += ksteps; }
  __device__ __forceinline__ void issue1(uint32_t lds_img, int wave, int kt, int n) {
    const int k0 = (kt + kt0) * BKT;  // wave-uniform: scalar math
    const int tap = k0 / g.C, cin0 = k0 - tap * g.C, kh = tap / g.KW, kw = tap - kh * g.KW;
    const int hi = ((int)hw[n] >> 16) + kh, wi = (int)(int16_t)(hw[n] & 0xffffu) + kw;
    const bool ok = (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
    const uint32_t voff = ok ? (uint32_t)(pix[n] + (kh * g.W + kw) * g.PP + cin0) * 2u : 0x80000000u;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_img + (n * NT + wave * 64) * 16);
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
                 "s"(dst)
                 : "memory");
  }
};

// Weight-gradient operand B = im2col(x) for dW = dyᵀ · im2col(x): GEMM K = output pixel
// (n, ho, wo), N = (kh, kw, c), staged as the M/N-contiguous image [64 pixels][256 columns]
// (chunk ^= mc_swz(k)). A thread's NDMA chunks share one image column (rows k, k+16, k+32,
// k+48 have equal mc_swz), hence one (kh, kw, c) for the whole kernel; each chunk walks its
// pixel forward by 64 per staged K-step (carry arithmetic, no divisions in the loop).
// Out-of-image taps read zeros through the buffer range check, as in ConvDmaA.
template <int NT, int NDMA>
struct ConvDmaBW {
  int base[NDMA];       // element offset of x[img][ho*S][wo*S][0] of the chunk's current pixel
  uint32_t hw[NDMA];    // ho << 16 | wo of that pixel
  int colterm;          // ((kh-P)*W + (kw-P))*C + c of the thread's column
  uint32_t kp;          // (kh-P) << 16 | (kw-P) & 0xffff
  u32x4 rs;
  ConvGeom g;
  int dH, dW;           // 64 pixels = dH output rows + dW output columns
  __device__ __forceinline__ void seek(int n, int pix) {
    const int wo = pix % g.Wo, t = pix / g.Wo, ho = t % g.Ho, im = t / g.Ho;
    base[n] = ((im * g.H + ho * g.S) * g.W + wo * g.S) * g.PP;
    hw[n] = ((uint32_t)ho << 16) | (uint32_t)wo;
  }
  __device__ __forceinline__ void init(const uint16_t* x, const ConvGeom& cg, int n0, int K, int tid) {
    g = cg;
    const int k = tid >> 5, c = (tid & 31) ^ mc_swz(k);  // same column for every chunk
    const int col = n0 + 8 * c;
    const int tap = col / g.C, cin = col - tap * g.C, kh = tap / g.KW, kw = tap - kh * g.KW;
    colterm = ((kh - g.P) * g.W + (kw - g.P)) * g.PP + cin;
    kp = ((uint32_t)(kh - g.P) << 16) | ((uint32_t)(kw - g.P) & 0xffffu);
    dH = 64 / g.Wo;
    dW = 64 - dH * g.Wo;
#pragma unroll
    for (int n = 0; n < NDMA; ++n) seek(n, (n * NT + tid) >> 5);
    const uint64_t b = (uint64_t)x;
    rs[0] = __builtin_amdgcn_readfirstlane((uint32_t)b);
    rs[1] = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) & 0xffffu;
    rs[2] = __builtin_amdgcn_readfirstlane((uint32_t)((int64_t)K / (g.Ho * g.Wo) * g.H * g.W * g.PP * 2));
    rs[3] = 0x00020000u;
  }
  __device__ __forceinline__ void advance(int ksteps) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int n = 0; n < NDMA; ++n) seek(n, ksteps * 64 + ((n * NT + tid) >> 5));
  }
  __device__ __forceinline__ void issue1(uint32_t lds_img, int wave, int /*kt*/, int n) {
    int ho = (int)(hw[n] >> 16), wo = (int)(hw[n] & 0xffffu);
    const int hi = ho * g.S + ((int)kp >> 16), wi = wo * g.S + (int)(int16_t)(kp & 0xffffu);
    const bool ok = (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
    const uint32_t voff = ok ? (uint32_t)(base[n] + colterm) * 2u : 0x80000000u;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_img + (n * NT + wave * 64) * 16);
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
                 "s"(dst)
                 : "memory");
    // this chunk's next staged K-step is 64 pixels further (carries, no divisions)
    const int SC = g.S * g.PP, SWC = g.S * g.W * g.PP;
    wo += dW;
    ho += dH;
    int b = base[n] + dW * SC + dH * SWC;
    if (wo >= g.Wo) { wo -= g.Wo; ho += 1; b += SWC - g.Wo * SC; }
    while (ho >= g.Ho) { ho -= g.Ho; b += g.H * g.W * g.PP - g.Ho * SWC; }
    base[n] = b;
    hw[n] = ((uint32_t)ho << 16) | (uint32_t)wo;
  }
};

// Fragment for rows [r0, r0+16) (row = lane&15), k = 32*s + 8*(lane>>4) + j of a K-step.
template <typename T, bool KC, int MCW = 256>
__device__ __forceinline__ typename V8<T>::type frag(const char* img, int r0, int s, int lane) {
  typedef typename V8<T>::type v8;
  if (KC) {
    const int row = r0 + (lane & 15), c = (4 * s + (lane >> 4)) ^ kc_swz(row);
    return *reinterpret_cast<const v8*>(img + row * 128 + c * 16);
  } else {
    // ds_read_b64_tr_b16: lane 4q+p of each 16-lane group g addresses k-row 32s+8g+q (+4),
    // columns r0+4p..+3, and receives its own column's 4 k-values.
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int k = 32 * s + 8 * g + q, x = mc_swz(k);  // mc_swz(k) == mc_swz(k + 4)
    const int c = ((r0 >> 3) + (p >> 1)) ^ x;
    const char* a0 = img + k * (2 * MCW) + c * 16 + 8 * (p & 1);
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a0);
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0 + 4 * (2 * MCW)));
    const u32x2 ul = __builtin_bit_cast(u32x2, lo), uh = __builtin_bit_cast(u32x2, hi);
    const u32x4 u = {ul[0], ul[1], uh[0], uh[1]};
    return __builtin_bit_cast(v8, u);
  }
}

// Second problem of a two-problem grouped launch (same M, K and layout; workgroups with a
// remapped id >= tiles1 run it): two weight gradients whose tile counts add up to one full wave
// of the chip (GPT-1.3B: qkv 192 + out-projection 64 = 256 tiles, one round of the full K loop
// instead of two split-K passes and their reductions).
struct GemmG2 {
  const uint16_t* A = nullptr;
  const uint16_t* B = nullptr;
  uint16_t* C = nullptr;
  int N = 0, lda = 0, ldb = 0, ldc = 0, tiles1 = 0;
};

template <typename T, typename CF, bool AK, bool BK, int E, bool BETA, bool SPLIT, bool CONV = false,
          int DPSX = 0, bool CONVW = false>
__global__ __launch_bounds__(CF::NT, 1) void gemm_lds_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
                                                          const uint16_t* __restrict__ bias, uint16_t* __restrict__ C,
                                                          uint16_t* __restrict__ Z, float* __restrict__ colsum,
                                                          int M, int N, int K, int lda, int ldb, int ldc, int ldz,
                                                          int splits, float* __restrict__ ws, ConvGeom cg = {},
                                                          float* __restrict__ colsq = nullptr,
                                                          const float* __restrict__ cshift = nullptr,
                                                          const uint8_t* __restrict__ mbits = nullptr,
                                                          GemmG2 g2 = {}) {
  constexpr int NT = CF::NT, TI = CF::TI, TJ = CF::TJ, NDA = CF::NDA, NDB = CF::NDB, WC = CF::WC;
  constexpr int BM = CF::BM, BN = CF::BN, IMGA = CF::IMGA, SLOT = CF::SLOT;
  constexpr int RW = TI * 16, CW = TJ * 16;  // rows / columns per wave
  static_assert(BK || BN == 256, "the M/N-contiguous B image is 256 columns wide");
  static_assert(AK || BM == 256 || BM == 128, "the M-contiguous A image is 256 or 128 columns wide");
  static_assert(!CONVW || (!BK && NDB == 4), "conv wgrad gathers the 256-wide B image");
  static_assert(TJ <= TI && 128 % RW == 0 && NDA >= 1 && NDB >= 1, "wave layout");
  __shared__ __attribute__((aligned(1024))) char lds[CF::LDS];
  typedef typename V8<T>::type v8;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  unsigned long long pra_tm[4] = {0, 0, 0, 0}, pra_ts[3] = {0, 0, 0};
  (void)pra_tm;
  (void)pra_ts;
  PRA_STAMP(0, __builtin_amdgcn_s_memtime());
  PRA_STAMP(4, __builtin_amdgcn_s_memrealtime());
  PRA_STAMP(6, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4));
  PRA_STAMP(7, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20));

  const int nb = gridDim.x;
  int pid = blockIdx.x;
  {  // contiguous tile run per XCD (bijective for any grid size)
    const int q = nb >> 3, r = nb & 7, xcd = pid & 7;
    pid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (pid >> 3);
  }
  if constexpr (!SPLIT && !CONV && !CONVW) {
    if (g2.tiles1 > 0 && pid >= g2.tiles1) {  // (wave-uniform: a whole workgroup switches)
      pid -= g2.tiles1;
      A = g2.A;
      B = g2.B;
      C = g2.C;
      N = g2.N;
      lda = g2.lda;
      ldb = g2.ldb;
      ldc = g2.ldc;
    }
  }
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  // split-K: the splits of one tile are adjacent ids (same XCD); each covers a K range and
  // writes an fp32 partial tile that splitk_reduce_k combines
  const int split = SPLIT ? pid % splits : 0;
  if (SPLIT) pid /= splits;
  const int group = 8 * tiles_n, gi = pid / group, first_m = gi * 8;
  const int gm = min(tiles_m - first_m, 8);
  const int tm = first_m + (pid % group) % gm, tn = (pid % group) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  // wave index as an SGPR value: the per-wave DMA destinations (M0) and fragment bases are then
  // scalar arithmetic (no v_readfirstlane + s_nop per LDS-DMA issue)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6),
            wr = wave / WC, wc = wave % WC;

  typename std::conditional<CONV, ConvDmaA<NT, NDA>, Dma<AK, NT, NDA, CF::BUF, (AK ? 256 : BM), CF::SC1>>::type da;
  typename std::conditional<CONVW, ConvDmaBW<NT, NDB>, Dma<BK, NT, NDB, CF::BUF, 256, CF::SC1>>::type db;
  if constexpr (CONV) da.init(A, cg, m0, M, tid);
  else if (AK) da.init(A, lda, m0, M - 1, tid);
  else da.init(A, lda, m0, M - 8, tid);
  if constexpr (CONVW) db.init(B, cg, n0, K, tid);
  else if (BK) db.init(B, ldb, n0, N - 1, tid);
  else db.init(B, ldb, n0, N - 8, tid);
  int nk = K / BKT;
  if (SPLIT) {
    const int per = (nk + splits - 1) / splits, kb = split * per;
    nk = max(0, min(nk, kb + per) - kb);
    da.advance(kb);
    db.advance(kb);
  }

  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  v8 fa0[TI], fb0[TJ], fa1[TI], fb1[TJ];
  constexpr bool AGPR_ACC = CF::WR * CF::WC == 4;  // 1 wave/SIMD: accumulators pinned to AGPRs
  auto read_frags = [&](v8 (&fa)[TI], v8 (&fb)[TJ], int kt, int s) __attribute__((always_inline)) {
    const char* ai = lds + (kt & 1) * SLOT;
    const char* bi = ai + IMGA;
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb[j] = frag<T, BK>(bi, wc * CW + j * 16, s, lane);
#pragma unroll
    for (int i = 0; i < TI; ++i) fa[i] = frag<T, AK, (AK ? 256 : BM)>(ai, wr * RW + i * 16, s, lane);
  };
  // 32 MFMAs of one k-half, interleaved segment by segment with (optionally) the fragment reads
  // of the next k-half and one LDS-DMA instruction of the next K-step every other segment, so
  // DMA issue and LDS reads hide under the wave's own matrix work.
  // dA / dB: issue this half's share of operand A's (step kA) / B's (step kB) DMA
  auto half = [&](v8 (&ca)[TI], v8 (&cb)[TJ], v8 (&na)[TI], v8 (&nb)[TJ], bool rd, int rkt, int rs, bool dA,
                  int kA, bool dB, int kB) __attribute__((always_inline)) {
    const uint32_t soA = lds_base + (kA & 1) * SLOT, soB = lds_base + (kB & 1) * SLOT + IMGA;
    const char* ai = lds + (rkt & 1) * SLOT;
    const char* bi = ai + IMGA;
    // DMA instructions per segment (DPSX > 0: front-load them into the first segments)
    constexpr int DPS = DPSX > 0 ? DPSX : (NDA + NDB + TI - 1) / TI;
    if constexpr (CF::ILV) {
      // segment i: MFMA j, then filler j -- the DMA pieces at even j, the two fragment reads at
      // j = 1, 3 -- each pinned in place, so the matrix pipe never waits behind a burst
#pragma unroll
      for (int i = 0; i < TI; ++i) {
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          if constexpr (AGPR_ACC) mma_agpr<T>(cb[j], ca[i], acc[i][j]);
          else acc[i][j] = mma<T>(cb[j], ca[i], acc[i][j]);
          __builtin_amdgcn_sched_barrier(0);
          if ((j & 1) == 0 && (j >> 1) < DPS && (dA || dB)) {
            const int d = i * DPS + (j >> 1);
            if (d < NDA) {
              if (dA) da.issue1(soA, wave, kA, d);
            } else if (d < NDA + NDB && dB) {
              db.issue1(soB, wave, kB, d - NDA);
            }
          } else if (j == 1 && rd && i < TJ) {
            nb[i] = frag<T, BK>(bi, wc * CW + i * 16, rs, lane);
          } else if (j == 3 && rd) {
            na[i] = frag<T, AK, (AK ? 256 : BM)>(ai, wr * RW + i * 16, rs, lane);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      if (dA || dB) {
#pragma unroll
        for (int d = i * DPS; d < (i + 1) * DPS && d < NDA + NDB; ++d) {
          if (d < NDA) {
            if (dA) da.issue1(soA, wave, kA, d);
          } else if (dB) {
            db.issue1(soB, wave, kB, d - NDA);
          }
        }
      }
      if (rd) {
        if (i < TJ) nb[i] = frag<T, BK>(bi, wc * CW + i * 16, rs, lane);
        na[i] = frag<T, AK, (AK ? 256 : BM)>(ai, wr * RW + i * 16, rs, lane);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        if constexpr (AGPR_ACC) mma_agpr<T>(cb[j], ca[i], acc[i][j]);
        else acc[i][j] = mma<T>(cb[j], ca[i], acc[i][j]);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // prologue: K-steps 0 and 1 in flight, k-half 0 of step 0 in registers
  if (nk > 0) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (t < nk) {
#pragma unroll
      for (int n = 0; n < NDA; ++n) da.issue1(lds_base + t * SLOT, wave, t, n);
#pragma unroll
      for (int n = 0; n < NDB; ++n) db.issue1(lds_base + t * SLOT + IMGA, wave, t, n);
    }
  }
  if (nk >= 2) {
    wait_vmcnt<NDA + NDB>();  // step 0 landed, step 1 still in flight
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  PRA_STAMP(1, __builtin_amdgcn_s_memtime());
  read_frags(fa0, fb0, 0, 0);

  // K-step kt (slot kt&1): half 0 computes (kt,0) from F0 while reading (kt,1) into F1; then the
  // barrier that retires step kt+1's DMA and every wave's reads of slot kt; half 1 refills slot kt
  // with step kt+2 (DMA) and computes (kt,1) from F1 while reading (kt+1,0) into F0.
  // (measured: issuing B of step kt+1 under half 0 of step kt instead, so both halves carry DMA,
  // was 8-15 % slower on every GPT shape: half a K-step does not cover the DMA latency)
  // (non-split launches pass splits = 0 only for the PRA_GEMM_ABLATE=nodma timing ablation)
  const bool dmaon = SPLIT || splits != 0;
  // STEADY: kt + 2 < nk and DMA on, known at compile time -> the K-step body has no branches
  // (the generic body tests "read next half" / "stage step kt+2" around every MFMA segment: ~16
  // wave-uniform branches per K-step in the steady state). The last two steps run the generic body.
  auto kstep = [&](int kt, auto steady_c) __attribute__((always_inline)) {
    constexpr bool STEADY = decltype(steady_c)::value;
    PRA_TMARK(0);
    half(fa0, fb0, fa1, fb1, true, kt, 1, false, 0, false, 0);
    __builtin_amdgcn_sched_barrier(0);
    PRA_TMARK(1);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): (kt,1) fragments landed; slot kt reads done
    if (STEADY || kt + 1 < nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // step kt+1 landed (this wave)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    PRA_TMARK(2);
    if constexpr (STEADY) {
      half(fa1, fb1, fa0, fb0, true, kt + 1, 0, true, kt + 2, true, kt + 2);
    } else {
      half(fa1, fb1, fa0, fb0, kt + 1 < nk, kt + 1, 0, kt + 2 < nk && dmaon, kt + 2, kt + 2 < nk && dmaon, kt + 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    PRA_TMARK(3);
    PRA_TACC();
    // (kt+1,0) fragments landed. The steady body leaves this to the compiler's per-register
    // lgkmcnt(N) before each consuming MFMA (no LDS-safety role: slot kt+1 is refilled only after
    // the next half-0 drain + barrier), so the next half starts on its first fragments.
    if constexpr (!STEADY) __builtin_amdgcn_s_waitcnt(0xC07F);
  };
  // PIPE schedule, K-step kt (slot kt&1):
  //   half 0: MFMAs of (kt,0) from F0; fillers = the reads of (kt,1) into F1, then lgkmcnt(0) +
  //           barrier A (every wave is done with slot kt), then the DMA refilling slot kt with
  //           step kt+2, one piece every other MFMA;
  //   vmcnt(pieces just issued) + barrier B: step kt+1 has landed for every wave;
  //   half 1: MFMAs of (kt,1) from F1; fillers = the reads of (kt+1,0) into F0.
  // A refill piece is consumed at half 1 of step kt+1: >= 2 k-halves after its issue.
  auto kstep_p = [&](int kt, auto steady_c) __attribute__((always_inline)) {
    constexpr bool STEADY = decltype(steady_c)::value;
    constexpr int NRD = TI + TJ, NDMA = NDA + NDB;
    static_assert(NRD + 1 + 2 * NDMA <= TI * TJ + 1, "PIPE: fillers exceed the half's MFMAs");
    const bool dma = STEADY || (kt + 2 < nk && dmaon);
    const bool rd1 = STEADY || kt + 1 < nk;
    {
      const char* ai = lds + (kt & 1) * SLOT;
      const char* bi = ai + IMGA;
      const uint32_t soA = lds_base + (kt & 1) * SLOT, soB = soA + IMGA;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          if constexpr (AGPR_ACC) mma_agpr<T>(fb0[j], fa0[i], acc[i][j]);
          else acc[i][j] = mma<T>(fb0[j], fa0[i], acc[i][j]);
          __builtin_amdgcn_sched_barrier(0);
          const int f = i * TJ + j;
          if (f < TJ) {
            fb1[f] = frag<T, BK>(bi, wc * CW + f * 16, 1, lane);
          } else if (f < NRD) {
            fa1[f - TJ] = frag<T, AK, (AK ? 256 : BM)>(ai, wr * RW + (f - TJ) * 16, 1, lane);
          } else if (f == NRD) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of slot kt done
            __builtin_amdgcn_s_barrier();        // barrier A: every wave's
          } else if (dma && ((f - NRD - 1) & 1) == 0 && (f - NRD - 1) / 2 < NDMA) {
            const int d = (f - NRD - 1) / 2;
            if (d < NDA) da.issue1(soA, wave, kt + 2, d);
            else db.issue1(soB, wave, kt + 2, d - NDA);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (dma) wait_vmcnt<NDA + NDB>();  // step kt+1's pieces landed (kt+2's may be in flight)
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // barrier B: step kt+1 landed for every wave
    __builtin_amdgcn_sched_barrier(0);
    {
      const char* ai = lds + ((kt + 1) & 1) * SLOT;
      const char* bi = ai + IMGA;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          if constexpr (AGPR_ACC) mma_agpr<T>(fb1[j], fa1[i], acc[i][j]);
          else acc[i][j] = mma<T>(fb1[j], fa1[i], acc[i][j]);
          __builtin_amdgcn_sched_barrier(0);
          const int f = i * TJ + j;
          if (rd1 && (f & 1) == 0 && f / 2 < NRD) {
            const int r = f / 2;
            if (r < TJ) fb0[r] = frag<T, BK>(bi, wc * CW + r * 16, 0, lane);
            else fa0[r - TJ] = frag<T, AK, (AK ? 256 : BM)>(ai, wr * RW + (r - TJ) * 16, 0, lane);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
    }
    if constexpr (!STEADY) __builtin_amdgcn_s_waitcnt(0xC07F);
  };
  // TS schedule, K-step kt (slot kt&1): one run of F = 2*NM MFMAs (NM = TI*TJ per k-half; the
  // first NM from F0 = (kt,0), the rest from F1 = (kt,1)), one filler slot after each MFMA f:
  //   f < NRD:        the reads of (kt,1) into F1 (slot kt is then fully in registers)
  //   f == BA:        lgkmcnt(0) + barrier: every wave is done with slot kt
  //   BA < f < BB:    the NDMA pieces of step kt+2 into slot kt, one every SP MFMAs (an LDS-DMA
  //                   issue needs ~60 cycles of MFMA cover; denser spacing stalls the matrix pipe)
  //   f == BB:        vmcnt(NDMA) (step kt+1 landed, kt+2 in flight) + barrier
  //   BB < f <= BB+NRD: the reads of (kt+1,0) into F0 (free since MFMA NM-1)
  // Every piece has ~1.5 K-steps of lead and no fragment read shares a stretch with DMA issue
  // (the loop shape of the 256x256x64 MFMA16 kernels hipBLASLt ships for gfx950).
  auto kstep_t = [&](int kt, auto steady_c) __attribute__((always_inline)) {
    constexpr bool STEADY = decltype(steady_c)::value;
    constexpr int NRD = TI + TJ, NDMA = NDA + NDB, NM = TI * TJ, F = 2 * NM;
    constexpr int BA = NRD + 4;                      // 20 of 128 (W4), 16 of 64 (W8)
    constexpr int BB = F - NRD - 3;                  // 109 (W4), 49 (W8)
    constexpr int SP = (BB - BA - 1) / NDMA > 0 ? (BB - BA - 1) / NDMA : 1;  // 5 (W4), 4 (W8)
    static_assert(BB >= NM && BA + 1 + (NDMA - 1) * SP < BB, "TS: fillers exceed the K-step's MFMAs");
    const bool dma = STEADY || (kt + 2 < nk && dmaon);
    const bool rd1 = STEADY || kt + 1 < nk;
    const uint32_t soA = lds_base + (kt & 1) * SLOT, soB = soA + IMGA;
    const char* ai = lds + (kt & 1) * SLOT;
    const char* bi = ai + IMGA;
    const char* an = lds + ((kt + 1) & 1) * SLOT;
    const char* bn = an + IMGA;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int f = h * NM + i * TJ + j;
      if (h == 0) {
        if constexpr (AGPR_ACC) mma_agpr<T>(fb0[j], fa0[i], acc[i][j]);
        else acc[i][j] = mma<T>(fb0[j], fa0[i], acc[i][j]);
      } else {
        if constexpr (AGPR_ACC) mma_agpr<T>(fb1[j], fa1[i], acc[i][j]);
        else acc[i][j] = mma<T>(fb1[j], fa1[i], acc[i][j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (f < TJ) {
        fb1[f] = frag<T, BK>(bi, wc * CW + f * 16, 1, lane);
      } else if (f < NRD) {
        fa1[f - TJ] = frag<T, AK, (AK ? 256 : BM)>(ai, wr * RW + (f - TJ) * 16, 1, lane);
      } else if (f == BA) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of slot kt done
        __builtin_amdgcn_s_barrier();        // every wave's
      } else if (f > BA && f < BB) {
        const int d = (f - BA - 1) / SP;
        if (dma && (f - BA - 1) % SP == 0 && d < NDMA) {
          if (d < NDA) da.issue1(soA, wave, kt + 2, d);
          else db.issue1(soB, wave, kt + 2, d - NDA);
        }
      } else if (f == BB) {
        if (dma) wait_vmcnt<NDMA>();  // step kt+1's pieces landed (kt+2's in flight)
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // ... for every wave
      } else if (rd1 && f > BB && f - BB - 1 < NRD) {
        const int r = f - BB - 1;
        if (r < TJ) fb0[r] = frag<T, BK>(bn, wc * CW + r * 16, 0, lane);
        else fa0[r - TJ] = frag<T, AK, (AK ? 256 : BM)>(an, wr * RW + (r - TJ) * 16, 0, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (!STEADY) __builtin_amdgcn_s_waitcnt(0xC07F);
  };
  if constexpr (CF::TS) {
    int kt = 0;
    if (dmaon)
      for (; kt + 2 < nk; ++kt) kstep_t(kt, std::true_type{});
    for (; kt < nk; ++kt) kstep_t(kt, std::false_type{});
  } else if constexpr (CF::PIPE) {
    int kt = 0;
    if (dmaon)
      for (; kt + 2 < nk; ++kt) kstep_p(kt, std::true_type{});
    for (; kt < nk; ++kt) kstep_p(kt, std::false_type{});
  } else {
  int kt = 0;
  // (the implicit-GEMM convolutions keep the generic body: their gather state already sits at
  // the register limit and a second body copy made them spill)
  if constexpr (!CONV && !CONVW)
    if (dmaon)
      for (; kt + 2 < nk; ++kt) kstep(kt, std::true_type{});
  for (; kt < nk; ++kt) kstep(kt, std::false_type{});
  }  // !PIPE
  }  // nk > 0
  PRA_STAMP(2, __builtin_amdgcn_s_memtime());
  PRA_STAMP(8, pra_ts[0]);
  PRA_STAMP(9, pra_ts[1]);
  PRA_STAMP(10, pra_ts[2]);

  // last asm MFMA -> v_accvgpr_read of its result: the hazard recognizer cannot see the asm
  if constexpr (AGPR_ACC) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  if (SPLIT) {
    float* wsp = ws + (int64_t)split * M * N;
    const int mrow = m0 + wr * RW + (lane & 15);
    const int ncol = n0 + wc * CW + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int m = mrow + i * 16;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int n = ncol + j * 16;
        if (n < N)
          *reinterpret_cast<float4*>(wsp + (int64_t)m * N + n) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }

  // Epilogue through LDS (the K loop is done with it): for each 128-row half the waves that own
  // it park their fp32 accumulators in an [128][256+4] image (ds_write_b128, conflict-free pitch),
  // then all 8 waves stream it out row-major: 8 columns per lane, whole 512-B row segments per 32
  // lanes, so the bias/activation/pre-activation/beta/dGELU traffic is 16-B coalesced loads and
  // stores instead of 8-B scatters across 16 rows.
  // acc[i][j][r] = C[m0 + wr*RW + i*16 + (lane&15)][n0 + wc*CW + j*16 + 4*(lane>>4) + r]
  float* img = reinterpret_cast<float*>(lds);
  constexpr int PITCH = BN + 4;  // floats
  // this thread's output units: row tid/TPR (+RSTEP per q), 8 columns at (tid%TPR)*8 (fixed per thread)
  constexpr int TPR = BN / 8, RSTEP = NT / TPR, NQ = 128 / RSTEP, QB = NQ < 4 ? NQ : 4;
  const int ucol = (tid % TPR) * 8, urow = tid / TPR;
  const int n = n0 + ucol;
  // output / Z / keep-bit row of GEMM row m (identity unless a strided-dgrad phase)
  auto orow = [&](int m) -> int64_t {
    if constexpr (CONV) {
      if (cg.OS) return (int64_t)cg.OS * cg.OS * m - (int64_t)cg.OS * (cg.OS - 1) * (m % cg.Wo);
    }
    return m;
  };
  const bool ncol_ok = n < N;  // N % 8 == 0: a unit is all-in or all-out
  float bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bv[e] = 0.f;
  if (bias && ncol_ok) {
    const uint4 bb = *reinterpret_cast<const uint4*>(bias + n);
    const uint32_t w4[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) { bv[2 * e] = to_f<T>(w4[e] & 0xffff); bv[2 * e + 1] = to_f<T>(w4[e] >> 16); }
  }
  // column statistics of the rounded output: colsum (bias gradient / BN sum) and, with colsq,
  // the sum of squares, both of (o - cshift[n]) when a shift is given (shifted-data variance)
  float cs[8], cq[8], ks[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { cs[e] = 0.f; cq[e] = 0.f; ks[e] = 0.f; }
  if (cshift && ncol_ok) {
#pragma unroll
    for (int e = 0; e < 8; ++e) ks[e] = cshift[n + e];
  }
  // kBnG with few units per thread (the narrow conv tiles): every Z / keep-bit load of the whole
  // epilogue is issued up front, so their latency overlaps the accumulator parking instead of
  // being paid once per 128-row chunk
  constexpr int NU = (BM / 128) * NQ;
  constexpr bool ZPRE = E == kBnG && NU <= 8;
  uint4 zp[ZPRE ? NU : 1];
  uint32_t mp[ZPRE ? NU : 1];
  if constexpr (ZPRE) {
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      const int m = m0 + (q / NQ) * 128 + urow + RSTEP * (q % NQ);
      if (m < M && ncol_ok) {
        const int64_t mo = orow(m);
        zp[q] = *reinterpret_cast<const uint4*>(Z + mo * ldz + n);
        mp[q] = mbits[(mo * N + n) >> 3];
      }
    }
  }
#pragma unroll
  for (int h = 0; h < BM / 128; ++h) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __syncthreads();  // (h=0) every wave is done reading K-loop tiles; (h>0) chunk h-1 streamed out
    if ((wr * RW) / 128 == h) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int r = wr * RW - h * 128 + i * 16 + (lane & 15), c = wc * CW + j * 16 + 4 * (lane >> 4);
          *reinterpret_cast<f32x4*>(img + r * PITCH + c) = acc[i][j];
        }
    }
    __syncthreads();
    // NQ units per thread in batches of 4: every load of a batch (LDS image, Z / C) is issued
    // before any of its math so the global-load latency is paid once per batch, not per unit
#pragma unroll
    for (int bq = 0; bq < NQ; bq += QB) {
      f32x4 lo[QB], hi[QB];
      uint4 gz[QB];
      uint32_t mb[QB];
      uint4 gc[(E == kBnG && BETA) ? QB : 1];   // kBnG + beta: the pending gradient C (added before the mask)
      bool ok[QB];
      int64_t moff[QB];
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        const int rr = urow + RSTEP * (bq + u), m = m0 + h * 128 + rr;
        ok[u] = m < M && ncol_ok;
        moff[u] = ok[u] ? orow(m) : 0;
        lo[u] = *reinterpret_cast<const f32x4*>(img + rr * PITCH + ucol);
        hi[u] = *reinterpret_cast<const f32x4*>(img + rr * PITCH + ucol + 4);
        if constexpr (E == kBnG && BETA) {
          if (ok[u]) gc[u] = *reinterpret_cast<const uint4*>(C + moff[u] * ldc + n);
        }
        if constexpr (ZPRE) {
          gz[u] = zp[h * NQ + bq + u];
          mb[u] = mp[h * NQ + bq + u];
        } else if (epi_scales(E) || E == kBnG) {
          if (ok[u]) gz[u] = *reinterpret_cast<const uint4*>(Z + moff[u] * ldz + n);
          if (E == kBnG && ok[u]) mb[u] = mbits[(moff[u] * N + n) >> 3];
        } else if (BETA) {
          if (ok[u]) gz[u] = *reinterpret_cast<const uint4*>(C + moff[u] * ldc + n);
        }
      }
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        if (!ok[u]) continue;
        const int64_t m = moff[u];
        float v[8] = {lo[u][0], lo[u][1], lo[u][2], lo[u][3], hi[u][0], hi[u][1], hi[u][2], hi[u][3]};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bv[e];
        if constexpr (epi_scales(E)) {
          const uint32_t w4[4] = {gz[u].x, gz[u].y, gz[u].z, gz[u].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float z0 = to_f<T>(w4[e] & 0xffff), z1 = to_f<T>(w4[e] >> 16);
            v[2 * e] *= zfac<E>(z0);
            v[2 * e + 1] *= zfac<E>(z1);
          }
        } else if constexpr (epi_gd(E)) {
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = act_d<E>(v[e], d[e]);
          uint4 o;
          o.x = pack2<T>(d[0], d[1]); o.y = pack2<T>(d[2], d[3]);
          o.z = pack2<T>(d[4], d[5]); o.w = pack2<T>(d[6], d[7]);
          *reinterpret_cast<uint4*>(Z + m * ldz + n) = o;
        } else if constexpr (E == kBnG) {
          if constexpr (BETA) {
            const uint32_t c4[4] = {gc[u].x, gc[u].y, gc[u].z, gc[u].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[2 * e] += to_f<T>(c4[e] & 0xffff); v[2 * e + 1] += to_f<T>(c4[e] >> 16); }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (mb[u] >> e) & 1u ? v[e] : 0.f;
        } else if (E != kNone) {
          if (Z) {
            uint4 o;
            o.x = pack2<T>(v[0], v[1]); o.y = pack2<T>(v[2], v[3]);
            o.z = pack2<T>(v[4], v[5]); o.w = pack2<T>(v[6], v[7]);
            *reinterpret_cast<uint4*>(Z + m * ldz + n) = o;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = act<E>(v[e]);
        }
        if (BETA && !epi_scales(E) && E != kBnG) {
          const uint32_t w4[4] = {gz[u].x, gz[u].y, gz[u].z, gz[u].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[2 * e] += to_f<T>(w4[e] & 0xffff); v[2 * e + 1] += to_f<T>(w4[e] >> 16); }
        }
        uint4 o;
        o.x = pack2<T>(v[0], v[1]); o.y = pack2<T>(v[2], v[3]);
        o.z = pack2<T>(v[4], v[5]); o.w = pack2<T>(v[6], v[7]);
        *reinterpret_cast<uint4*>(C + m * ldc + n) = o;
        if (colsum) {
          // the bias gradient sums the ROUNDED output (what a separate reduction would read)
          const uint32_t w4[4] = {o.x, o.y, o.z, o.w};
          if constexpr (E == kBnG) {
            const uint32_t z4[4] = {gz[u].x, gz[u].y, gz[u].z, gz[u].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float g0 = to_f<T>(w4[e] & 0xffff), g1 = to_f<T>(w4[e] >> 16);
              cs[2 * e] += g0;
              cs[2 * e + 1] += g1;
              cq[2 * e] += g0 * (to_f<T>(z4[e] & 0xffff) - ks[2 * e]);
              cq[2 * e + 1] += g1 * (to_f<T>(z4[e] >> 16) - ks[2 * e + 1]);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float d0 = to_f<T>(w4[e] & 0xffff) - ks[2 * e], d1 = to_f<T>(w4[e] >> 16) - ks[2 * e + 1];
              cs[2 * e] += d0;
              cs[2 * e + 1] += d1;
              if (colsq) { cq[2 * e] += d0 * d0; cq[2 * e + 1] += d1 * d1; }
            }
          }
        }
      }
    }
  }
  if (colsum) {
    // threads with equal tid % TPR own the same 8 columns: reduce over the lanes l, l + TPR, ...
    // of each wave, then over the waves through LDS (one 8-column group per lane < TPR)
#pragma unroll
    for (int o = TPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[e] += __shfl_xor(cs[e], o, 64);
        if (colsq) cq[e] += __shfl_xor(cq[e], o, 64);
      }
    __syncthreads();
    if (lane < TPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        img[wave * BN + lane * 8 + e] = cs[e];
        if (colsq) img[(NT / 64 + wave) * BN + lane * 8 + e] = cq[e];
      }
    }
    __syncthreads();
    for (int t = tid; t < BN; t += NT) {
      float a = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) {
        a += img[w * BN + t];
        if (colsq) q += img[(NT / 64 + w) * BN + t];
      }
      const int nn = n0 + t;
      if (nn < N) {
        colsum[(int64_t)tm * N + nn] = a;
        if (colsq) colsq[(int64_t)tm * N + nn] = q;
      }
    }
  }
  if constexpr (PRA_GEMM_STAMPS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PRA_STAMP(3, __builtin_amdgcn_s_memtime());
  PRA_STAMP(5, __builtin_amdgcn_s_memrealtime());
}

// split-K combine: C[m][n..n+3] = epi(sum_s ws[s][m][n..n+3] + bias) (+ C if BETA).
// G (power of two, <= 256) lanes per 4-column quad: lane g sums splits g, g+G, ... (4 loads in
// flight), then the G partials are added in lane order through LDS. G > 1 for small outputs
// with many splits (a ResNet 1x1 weight gradient: 64 x 256 outputs, 256 splits), which with one
// lane per quad ran 4-32 workgroups of 256 dependent loads each (splitk_groups picks G).
// G = 1 keeps the plain split order.
template <typename T, int E, bool BETA>
__global__ void __launch_bounds__(256) splitk_reduce_k(const float* __restrict__ ws, int splits,
                                                       const uint16_t* __restrict__ bias, uint16_t* __restrict__ C,
                                                       uint16_t* __restrict__ Z, int M, int N, int ldc, int ldz,
                                                       int G = 1) {
  __shared__ float4 red[256];
  const int g = threadIdx.x & (G - 1);
  const int64_t MN = (int64_t)M * N;
  const int64_t idx = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G) * 4;
  const bool valid = idx < MN;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid) {
    int s = g;
    for (; s + 3 * G < splits; s += 4 * G) {
      float4 b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) b[u] = *reinterpret_cast<const float4*>(ws + (int64_t)(s + u * G) * MN + idx);
#pragma unroll
      for (int u = 0; u < 4; ++u) { a.x += b[u].x; a.y += b[u].y; a.z += b[u].z; a.w += b[u].w; }
    }
    for (; s < splits; s += G) {
      const float4 b = *reinterpret_cast<const float4*>(ws + (int64_t)s * MN + idx);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  if (G > 1) {
    red[threadIdx.x] = a;
    __syncthreads();
    if (g != 0) return;   // (no barrier after this point)
    for (int j = 1; j < G; ++j) {
      const float4 b = red[threadIdx.x + j];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  if (!valid) return;
  const int m = (int)(idx / N), n = (int)(idx % N);
  float v[4] = {a.x, a.y, a.z, a.w};
  if (bias) {
    const uint2 bb = *reinterpret_cast<const uint2*>(bias + n);
    v[0] += to_f<T>(bb.x & 0xffff); v[1] += to_f<T>(bb.x >> 16);
    v[2] += to_f<T>(bb.y & 0xffff); v[3] += to_f<T>(bb.y >> 16);
  }
  if constexpr (epi_gd(E)) {
    float d[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = act_d<E>(v[r], d[r]);
    uint2 o;
    o.x = pack2<T>(d[0], d[1]);
    o.y = pack2<T>(d[2], d[3]);
    *reinterpret_cast<uint2*>(Z + (int64_t)m * ldz + n) = o;
  } else if (E != kNone) {
    if (Z) {
      uint2 o;
      o.x = pack2<T>(v[0], v[1]);
      o.y = pack2<T>(v[2], v[3]);
      *reinterpret_cast<uint2*>(Z + (int64_t)m * ldz + n) = o;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = act<E>(v[r]);
  }
  uint16_t* c = C + (int64_t)m * ldc + n;
  if (BETA) {
    const uint2 cc = *reinterpret_cast<const uint2*>(c);
    v[0] += to_f<T>(cc.x & 0xffff); v[1] += to_f<T>(cc.x >> 16);
    v[2] += to_f<T>(cc.y & 0xffff); v[3] += to_f<T>(cc.y >> 16);
  }
  uint2 o;
  o.x = pack2<T>(v[0], v[1]);
  o.y = pack2<T>(v[2], v[3]);
  *reinterpret_cast<uint2*>(c) = o;
}

// sum of P partial rows [P][N] fp32 -> out[N] (dtype T)
template <typename T>
__global__ void colsum_partials_k(const float* __restrict__ part, T* __restrict__ out, int P, int N) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += part[(int64_t)p * N + n];
  out[n] = Cvt<T>::from(s);
}

}  // namespace
}  // namespace pra
