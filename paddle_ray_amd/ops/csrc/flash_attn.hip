// Flash attention forward + backward for gfx950 (CDNA4) on v_mfma_f32_32x32x16_{bf16,f16}.
//
// Layout: q,k,v,o are [B, S, H, D] with D contiguous (arbitrary b/s/h strides so
// the GPT fused-QKV projection output is consumed in place); lse/delta are
// [B, H, S] fp32. D in {64, 128}.
//
// "Swapped" formulation (CDNA4 guide §3 'accumulator as next operand', T12):
//   S^T = K Q^T  -> the 32x32 accumulator holds one QUERY per lane (column),
//                   keys in registers: softmax row stats are lane-local
//                   (one __shfl_xor(.,32) for the row max/sum).
//   O^T += V^T P^T -> P^T's accumulator registers ARE the B operand (k order
//                   permuted: elem j of lane-half h <-> key 16s+8(j>>2)+4h+(j&3)),
//                   V^T comes from the same swizzled V tile image through
//                   ds_read_b64_tr_b16 (hardware transposed read, guide T10).
//                   The O^T accumulator is again one query per lane, so the
//                   online-softmax rescale is lane-local too.
// Backward = FA2 split into a dK/dV kernel (keys on lanes, sweep queries) and a
// dQ kernel (queries on lanes, sweep keys): no float atomics (MI355X atomics
// are ~1.3 TB/s chip-wide; dQ atomics would cost more than the whole backward).
//
// Tiles of 64 rows (K/V in fwd and dQ, Q/dO in dK/dV) are staged ONCE per tile into a
// swizzled LDS image (8x32 subtiles, XOR chunk swizzle) that serves both row fragments
// (ds_read_b128) and transposed fragments; two LDS buffers alternate so the next tile is
// written right after the current tile's MFMAs (one barrier per tile), with its global
// loads issued at the top of the iteration (async-STAGE split, guide T14).
// fwd / dQ: 8 waves, 32 queries per wave (2 waves per SIMD); dK/dV: 4 waves, 32 keys per
// wave (one wave per SIMD, 256 + accumulator registers).
#include "common.h"
#include <stdlib.h>
#include <string.h>
#include <type_traits>
#include <algorithm>
#include <cmath>

namespace pra {
namespace fa {

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// s_waitcnt vmcnt(0) (expcnt/lgkmcnt left at max). Placed right after the per-wave
// register fragments are loaded in the prologue: without it the waitcnt pass cannot prove
// at the loop header that those prologue loads retired and puts a vmcnt(0) in front of the
// FIRST MFMA of every iteration -- which then also waits for the NEXT tile's prefetch.
__device__ __forceinline__ void wait_vmem_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <typename T> struct V8;
template <> struct V8<bf16> { typedef __bf16 type __attribute__((ext_vector_type(8))); };
template <> struct V8<f16> { typedef _Float16 type __attribute__((ext_vector_type(8))); };

template <typename T>
__device__ __forceinline__ f32x16 mfma(typename V8<T>::type a, typename V8<T>::type b, f32x16 c);
template <>
__device__ __forceinline__ f32x16 mfma<bf16>(V8<bf16>::type a, V8<bf16>::type b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x16 mfma<f16>(V8<f16>::type a, V8<f16>::type b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <typename T> __device__ __forceinline__ uint32_t pack2(float a, float b);
template <> __device__ __forceinline__ uint32_t pack2<bf16>(float a, float b) { return pack_bf2(a, b); }
template <> __device__ __forceinline__ uint32_t pack2<f16>(float a, float b) {
  _Float16 x = (_Float16)a, y = (_Float16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}
template <typename T> __device__ __forceinline__ float lo16(uint32_t w);
template <typename T> __device__ __forceinline__ float hi16(uint32_t w);
template <> __device__ __forceinline__ float lo16<bf16>(uint32_t w) { return __uint_as_float(w << 16); }
template <> __device__ __forceinline__ float hi16<bf16>(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
template <> __device__ __forceinline__ float lo16<f16>(uint32_t w) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffff));
}
template <> __device__ __forceinline__ float hi16<f16>(uint32_t w) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
}

template <typename T>
__device__ __forceinline__ typename V8<T>::type as_v8(u32x4 u) {
  return __builtin_bit_cast(typename V8<T>::type, u);
}
// 8 accumulator registers (floats) -> one MFMA operand fragment
template <typename T>
__device__ __forceinline__ typename V8<T>::type pack_frag(const f32x16& acc, int base) {
  u32x4 u;
  u[0] = pack2<T>(acc[base + 0], acc[base + 1]);
  u[1] = pack2<T>(acc[base + 2], acc[base + 3]);
  u[2] = pack2<T>(acc[base + 4], acc[base + 5]);
  u[3] = pack2<T>(acc[base + 6], acc[base + 7]);
  return as_v8<T>(u);
}

constexpr int kTile = 64;        // rows per staged tile (keys in fwd/dQ, queries in dK/dV)

// Extended attention (the EXT kernel variants; parity: flash_attn_kernel.cu:183 / :250 and
// python/paddle/nn/functional/flash_attention.py:20,121):
//   * varlen (flash_attn_unpadded): q/k/v/o rows packed [total, H, D]; sequence b is rows
//     [cu_q[b], cu_q[b+1]) of q/o and [cu_k[b], cu_k[b+1]) of k/v. lse / delta stay
//     [B, H, SqMax] (padded), the dS^T scratch [B*H][SkMax][SqMax] (rounded).
//   * additive mask [B|1, H|1, Sq, Sk] (element strides msb/msh/msq, 0 = broadcast; keys
//     contiguous), in q's dtype or fp32, added to the scaled scores.
//   * dropout on the probabilities: keep iff a counter hash of (seed, offset, b*H+h, query, key)
//     clears the threshold; kept values scaled by 1/(1-p). The backward regenerates the same
//     bits (FA2: dV = (P∘Z)ᵀdO, dS = P∘(Z∘dP − delta), delta = rowsum(dO∘O)).
struct FaExt {
  const int* cu_q;
  const int* cu_k;
  const void* mask;
  int64_t msb, msh, msq;
  int mask_f32;
  float mask_mul;  // 1 / scale: the kernels add mask/scale to the raw q·k scores
  uint32_t thr;    // dropout threshold on 16-bit uniforms, round(p * 65536) (0 = no dropout)
  float inv_keep;  // 65536 / (65536 - thr)
  uint64_t seed, offset;
  // dropout keep bits the forward stores for the backward: [B*H][SqMax][dbits_ld] words, bit
  // (key & 31) of word (query, key >> 5); the dK/dV kernel reads them instead of re-hashing
  uint32_t* dbits;
  int dbits_ld;
  int xf;  // feature set of the launch (XF_* below), chosen on the host
  // graph replays: device step counter mixed into the seed (null in eager launches; see
  // ops/graph_rng.py): a captured launch draws new bits on every replay
  const uint64_t* dseq;
  // packed-QKV bias gradient (Sq == Sk, no varlen): column-sum partials of the rounded dQ / dK / dV,
  // one fp32 row per (batch, 128-row block): bsum[(b * bsum_nblk + blk) * 3HD + which * HD + h * D + d]
  // (which = 0 / 1 / 2 for q / k / v), reduced into the bias gradient by colsum16(_acc)
  float* bsum;
  int bsum_nblk;
};

// Feature bits of an extended launch. Each combination runs its own copy of the tile loop, so
// a feature that is off costs nothing inside the loop (runtime tests of ext.mask / ext.thr per
// score element split the MFMA/VALU schedule: the extended kernels without extras ran 20 %
// (fwd) / 42 % (bwd) slower than the plain ones at BERT-base shapes).
//   XF_DROP : dropout on the probabilities
//   XF_KMASK: additive mask that depends on the key only (msq == 0: [B|1, H|1, 1, Sk], the
//             padding mask of BERT-style encoders): fwd stages the block's mask row in LDS once,
//             dK/dV holds its lane's key value in a register
//   XF_FMASK: general [B|1, H|1, Sq, Sk] mask, read per score element
enum : int { XF_DROP = 1, XF_KMASK = 2, XF_FMASK = 4 };

__device__ __forceinline__ uint32_t fa_mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
// Dropout keep decision of element (query q, key kk) of head row bh. One lowbias32 round over a
// multiply-xor fold of (seed, offset, bh, q, kk >> 1) yields the 16-bit uniforms of a PAIR of
// adjacent keys (low half: even key, high half: odd key): one hash per two scores, against one
// per score before (the two 32-bit multiplies of the mix are quarter-rate VALU and were the
// dominant cost of dropout at head_dim 64). keep iff u16 >= thr (thr = round(p * 65536): the
// dropout rate is p to within 2^-17, kept values scaled by the exact 1/(1-thr/65536)). fwd and
// bwd call the same function, so a backward without stored bits regenerates them exactly.
__device__ __forceinline__ uint32_t fa_key(const FaExt& e, int bh) {
  const uint64_t seed = e.dseq ? e.seed ^ (*e.dseq * 0x9E3779B97F4A7C15ull) : e.seed;
  return fa_mix32((uint32_t)seed ^ (uint32_t)(seed >> 32) * 0x27d4eb2fU ^
                  (uint32_t)e.offset * 0x165667b1U ^ (uint32_t)bh * 0xc2b2ae3dU);
}
__device__ __forceinline__ uint32_t fa_hash2(uint32_t key, int q, int kpair) {
  return fa_mix32(key ^ (uint32_t)q * 0x9e3779b1U ^ (uint32_t)kpair * 0x85ebca77U);
}
__device__ __forceinline__ float fa_keep(const FaExt& e, uint32_t u16) { return u16 >= e.thr ? e.inv_keep : 0.f; }
__device__ __forceinline__ float fa_drop(const FaExt& e, uint32_t key, int q, int kk) {
  const uint32_t hs = fa_hash2(key, q, kk >> 1);
  return fa_keep(e, (kk & 1) ? (hs >> 16) : (hs & 0xffffu));
}
// additive mask value (already divided by the softmax scale) of (b, h, query q, key kk)
template <typename T>
__device__ __forceinline__ float fa_mask(const FaExt& e, int b, int hh, int q, int kk) {
  const int64_t i = (int64_t)b * e.msb + (int64_t)hh * e.msh + (int64_t)q * e.msq + kk;
  float m;
  if (e.mask_f32) m = static_cast<const float*>(e.mask)[i];
  else m = Cvt<T>::to(static_cast<const T*>(e.mask)[i]);
  return m * e.mask_mul;
}

// Swizzled tile image [64][D] (no padding), element offset of 16-B chunk ch of row `row`:
// 8-row x 32-column subtiles of 512 B, chunk (ch&3) XOR-ed with (row>>2)&3. One image serves
// row fragments (ds_read_b128) and transposed fragments (ds_read_b64_tr_b16) bank-conflict
// free, and the reads of one fragment set differ by immediates from 2 base registers.
template <int D>
__device__ __forceinline__ int swz(int row, int ch) {
  return (row >> 3) * (8 * D) + (ch >> 2) * 256 + (row & 7) * 32 + 8 * ((ch & 3) ^ ((row >> 2) & 3));
}

// Block-cooperative staged load of a 64-row x D tile by NT threads, row-coalesced mapping:
// chunk c = t + NT*p -> row c / NCH, 16-B column chunk c % NCH, so consecutive lanes read
// consecutive 16 B of the same row and one wave instruction touches 64*16/NCH... whole
// 128-B lines (D=128: 4 rows x 256 B) instead of 16-B pieces of 64 different rows (which
// left the texture-address unit stalled on 64 partial lines per instruction).
template <typename T, int D, int NT>
struct TileRegs {
  static constexpr int NCH = D / 8;                          // 16-B chunks per row
  static constexpr int NPASS = (kTile * NCH + NT - 1) / NT;
  uint4 r[NPASS];

  __device__ __forceinline__ void load(const T* base, int64_t row_stride, int row0, int nrows) {
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int c = threadIdx.x + NT * p, row = c / NCH, dc = c % NCH;
      const int rr = row0 + row;
      r[p] = (row < kTile && rr < nrows)
                 ? *reinterpret_cast<const uint4*>(base + (int64_t)rr * row_stride + dc * 8)
                 : make_uint4(0, 0, 0, 0);
    }
  }
  // swizzled row image [64][D] (see swz)
  __device__ __forceinline__ void store_swz(T* img) const {
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int c = threadIdx.x + NT * p, row = c / NCH, dc = c % NCH;
      if (row < kTile) *reinterpret_cast<uint4*>(img + swz<D>(row, dc)) = r[p];
    }
  }
};

// operand fragment straight from global (row pointer + d offset), zero if invalid
template <typename T>
__device__ __forceinline__ typename V8<T>::type frag_global(const T* rowp, int d, bool valid) {
  u32x4 u = {0, 0, 0, 0};
  if (valid) {
    uint4 x = *reinterpret_cast<const uint4*>(rowp + d);
    u[0] = x.x; u[1] = x.y; u[2] = x.z; u[3] = x.w;
  }
  return as_v8<T>(u);
}

__device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
// Per-lane element offsets into a swizzled [64][D] image, computed ONCE per kernel: every
// row / transposed fragment is then (image base + lane offset + compile-time immediate), so
// the tile loops carry no per-fragment address arithmetic (swz() with runtime lane terms
// cost ~100 VALU per tile). Derivation: for row = 32*mt + r and chunk 2s+h, swz() splits into
// mt*32D + (s>>1)*256 + [lane part depending on s&1]; for the transposed read of k-step S,
// d-tile dt it is S*16D + dt*256 + [lane part], with a second lane part for rows +8.
template <int D>
struct LaneOffs {
  int row[2];
  int tra, trb;
  __device__ __forceinline__ explicit LaneOffs(int lane) {
    const int r = lane & 31, h = lane >> 5, x = (r >> 2) & 3;
    row[0] = (r >> 3) * 8 * D + (r & 7) * 32 + 8 * (h ^ x);
    row[1] = (r >> 3) * 8 * D + (r & 7) * 32 + 8 * ((2 + h) ^ x);
    const int g = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    const int cc = 2 * g + (p >> 1);
    tra = (4 * h + q) * 32 + 8 * (cc ^ h) + 4 * (p & 1);
    trb = 8 * D + (4 * h + q) * 32 + 8 * (cc ^ (h + 2)) + 4 * (p & 1);
  }
};

// row fragment of image rows 32*mt + (lane&31), k-step s: 16 B of row at chunk 2s+h
template <typename T, int D>
__device__ __forceinline__ typename V8<T>::type frag_rows(const T* img, const LaneOffs<D>& lo, int mt, int s) {
  return *reinterpret_cast<const typename V8<T>::type*>(img + lo.row[s & 1] + mt * 32 * D + (s >> 1) * 256);
}

// Transposed A fragment (row = column 32*dt + (lane&31) of the image) over the k-step S of
// the image's rows, in the permuted k order of an accumulator-derived B operand:
// elem j <-> image row 16S + 8(j>>2) + 4h + (j&3). Two ds_read_b64_tr_b16: lane 4q+p of each
// 16-lane group addresses row (base+q), columns 4p..4p+3 of the group's 16 columns and
// receives its own column of the 4 rows. EXEC must be full (every lane takes part).
template <typename T, int D>
__device__ __forceinline__ typename V8<T>::type frag_tr(const T* img, const LaneOffs<D>& lo, int dt, int S) {
  const T* pa = img + lo.tra + S * 16 * D + dt * 256;
  const T* pb = img + lo.trb + S * 16 * D + dt * 256;
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)pa);
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)pb);
  const u32x2 ua = __builtin_bit_cast(u32x2, a), ub = __builtin_bit_cast(u32x2, b);
  u32x4 u;
  u[0] = ua[0]; u[1] = ua[1]; u[2] = ub[0]; u[3] = ub[1];
  return as_v8<T>(u);
}

// LDS-DMA plan for one swizzled [64][W] image (W = row length in elements): DMA instruction n of
// a wave writes image elements [512 (n*NWV + wave), +512), lane l the 8 at +8l. Per lane the
// (row, chunk) that lands there, as a byte offset from the tile's first row.
template <int W, int NT>
struct SwzDma {
  static constexpr int NI = kTile * W * 2 / 1024;  // 1-KB DMA instructions per tile
  static constexpr int PER = NI / (NT / 64);       // per wave
  static_assert(NI % (NT / 64) == 0, "DMA split");
  uint32_t voff[PER];
  u32x4 rs;
  __device__ __forceinline__ void init(const void* base, int64_t pitch_el, int nrows, int wave, int lane) {
#pragma unroll
    for (int n = 0; n < PER; ++n) {
      const int E = 512 * (n * (NT / 64) + wave) + 8 * lane;  // image element offset
      const int rg = E / (8 * W), rem = E % (8 * W), cg = rem / 256, r2 = rem % 256;
      const int row = rg * 8 + r2 / 32, x = (r2 % 32) / 8;
      const int ch = cg * 4 + (x ^ ((row >> 2) & 3));
      voff[n] = (uint32_t)((row * pitch_el + ch * 8) * 2);
    }
    const uint64_t bb = (uint64_t)base;
    rs[0] = __builtin_amdgcn_readfirstlane((uint32_t)bb);
    rs[1] = __builtin_amdgcn_readfirstlane((uint32_t)(bb >> 32)) & 0xffffu;  // stride 0
    rs[2] = __builtin_amdgcn_readfirstlane((uint32_t)((int64_t)nrows * pitch_el * 2));  // rows >= nrows read 0
    rs[3] = 0x00020000u;
  }
  // stage the tile whose first row is at byte offset row_bytes into the image at LDS byte address img
  __device__ __forceinline__ void issue(uint32_t img, uint32_t row_bytes, int wave) {
    // the descriptor is wave-uniform, but the copies of the tile loop behind a switch on the
    // feature set can leave it in VGPRs: pin it to SGPRs for the "s" constraint
    const u32x4 srs = {(uint32_t)__builtin_amdgcn_readfirstlane(rs[0]), (uint32_t)__builtin_amdgcn_readfirstlane(rs[1]),
                       (uint32_t)__builtin_amdgcn_readfirstlane(rs[2]), (uint32_t)__builtin_amdgcn_readfirstlane(rs[3])};
#pragma unroll
    for (int n = 0; n < PER; ++n) {
      const uint32_t dst = __builtin_amdgcn_readfirstlane(img + 1024u * (n * (NT / 64) + wave));
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff[n] + row_bytes),
                   "s"(srs), "s"(dst)
                   : "memory", "m0");
    }
  }
};

// One 4-byte-per-lane LDS-DMA: lane l's dword at byte offset voff of the buffer rs lands at LDS
// byte dst + 4*l (offsets past the descriptor's range read 0). Issued from asm like SwzDma, so the
// compiler's waitcnt model never sees it: the loops' explicit counted vmcnt are its only waits.
__device__ __forceinline__ void dma_dword(const u32x4& rs, uint32_t voff, uint32_t dst) {
  const u32x4 srs = {(uint32_t)__builtin_amdgcn_readfirstlane(rs[0]), (uint32_t)__builtin_amdgcn_readfirstlane(rs[1]),
                     (uint32_t)__builtin_amdgcn_readfirstlane(rs[2]), (uint32_t)__builtin_amdgcn_readfirstlane(rs[3])};
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds" ::"v"(voff), "s"(srs),
               "s"(__builtin_amdgcn_readfirstlane(dst))
               : "memory", "m0");
}
__device__ __forceinline__ u32x4 raw_desc(const void* base, uint64_t bytes) {
  const uint64_t bb = (uint64_t)base;
  return u32x4{(uint32_t)bb, (uint32_t)(bb >> 32) & 0xffffu, (uint32_t)bytes, 0x00020000u};
}
// s_waitcnt vmcnt(N), other counters unconstrained
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

// ============================================================================
// forward
// ============================================================================
template <typename T, int D, bool CAUSAL, int NW, bool EXT = false>
__global__ void __launch_bounds__(NW * 64, 2)
fwd_kernel(const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, T* __restrict__ o,
           float* __restrict__ lse, int H, int SqM, int SkM, int64_t qsb, int64_t qss, int64_t qsh, int64_t ksb,
           int64_t kss, int64_t ksh, int64_t vsb, int64_t vss, int64_t vsh, float scale_log2, FaExt ext = {}) {
  // double-buffered {K, V} swizzled images; V^T fragments by transposed reads of V
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* img0 = reinterpret_cast<T*>(smem);  // [2][2][64*D]
  constexpr int NS = D / 16, ND = D / 32, BM = NW * 32;

  const int nqb = gridDim.y;
  // grid (B*H, q-blocks): every (b, h) of one q-block row launches before the next row, so
  // the heaviest causal blocks of ALL heads go first (LPT order, no late 16-tile straggler),
  // and the q-blocks of one head share an XCD's L2 for K/V when B*H % 8 == 0
  const int qb = CAUSAL ? (nqb - 1 - blockIdx.y) : blockIdx.y;
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int q0 = qb * BM;
  const int myq = q0 + wave * 32 + r;
  int Sq = SqM, Sk = SkM;
  int64_t qrow0 = (int64_t)b * SqM, krow0 = 0;  // first packed row of this sequence (o rows / k,v rows)
  if constexpr (EXT) {
    if (ext.cu_q) {
      qrow0 = ext.cu_q[b];
      krow0 = ext.cu_k[b];
      Sq = ext.cu_q[b + 1] - (int)qrow0;
      Sk = ext.cu_k[b + 1] - (int)krow0;
      if (q0 >= Sq) return;  // the whole block is past this sequence (uniform: before any barrier)
    }
  }
  const int off = Sk - Sq;
  const uint32_t dkey = EXT ? fa_key(ext, bh) : 0u;  // per-(head row) dropout hash key

  const T* qb_ = EXT && ext.cu_q ? q + qrow0 * qss + hh * qsh : q + b * qsb + hh * qsh;
  const T* kb_ = EXT && ext.cu_q ? k + krow0 * kss + hh * ksh : k + b * ksb + hh * ksh;
  const T* vb_ = EXT && ext.cu_q ? v + krow0 * vss + hh * vsh : v + b * vsb + hh * vsh;

  typename V8<T>::type qf[NS];
  {
    const bool valid = myq < Sq;
    const T* rowp = qb_ + (int64_t)(valid ? myq : 0) * qss;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = frag_global<T>(rowp, 16 * s + 8 * h, valid);
  }
  // (no wait here: the Q fragment loads stay in flight under the first K/V tile's DMA below and
  // are retired by the same vmcnt(0) before the first barrier -- one HBM round trip per block
  // prologue instead of two; causal blocks at S = 1024 sweep only 2-16 tiles)

  f32x16 acc_o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) acc_o[i] = f32x16{};
  float m_run = -INFINITY, l_run = 0.f;  // m in the scaled log2 domain

  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, q0 + BM + off);
  const int ntiles = n_end > 0 ? (n_end + kTile - 1) / kTile : 0;

  // K/V tiles are staged by LDS-DMA straight into the swizzled images (no VGPR staging and no
  // ds_write; the buffer range check zero-fills key rows >= Sk)
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  SwzDma<D, NW * 64> kd, vd;
  kd.init(kb_, kss, Sk, wave, lane);
  vd.init(vb_, vss, Sk, wave, lane);
  auto stage = [&](int kt) {
    const uint32_t img = lds0 + (uint32_t)((2 * (kt & 1)) * kTile * D * sizeof(T));
    kd.issue(img, (uint32_t)((int64_t)kt * kTile * kss * 2), wave);
    vd.issue(img + kTile * D * sizeof(T), (uint32_t)((int64_t)kt * kTile * vss * 2), wave);
  };
  if (ntiles > 0) stage(0);
  // XF_KMASK: this (b, h)'s mask row, pre-multiplied by mask_mul, in LDS behind the K/V images
  // (keys past Sk read 0; the launcher sizes the LDS to the 64-rounded Sk)
  float* mrow = reinterpret_cast<float*>(smem + 4 * kTile * D * sizeof(T));
  if constexpr (EXT) {
    if (ext.xf & XF_KMASK) {
      const int64_t mb = (int64_t)b * ext.msb + (int64_t)hh * ext.msh;
      for (int j = threadIdx.x; j < ntiles * kTile; j += NW * 64) {
        float m = 0.f;
        if (j < Sk) {
          m = ext.mask_f32 ? static_cast<const float*>(ext.mask)[mb + j]
                           : Cvt<T>::to(static_cast<const T*>(ext.mask)[mb + j]);
          m *= ext.mask_mul;
        }
        mrow[j] = m;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const LaneOffs<D> lo(lane);
  // one tile: the masked variant only for tiles that straddle Sk or the causal diagonal; XF =
  // the extended features compiled into this copy of the loop
  auto tile = [&](int kt, auto mask_c, auto xf_c) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(mask_c)::value;
    constexpr int XF = decltype(xf_c)::value;
    const int k0 = kt * kTile;
    const T* Ks = img0 + (2 * (kt & 1)) * kTile * D;
    const T* Vs = Ks + kTile * D;
    if (kt + 1 < ntiles) stage(kt + 1);  // idle buffer: last read before the previous barrier
    // masked tiles: 32-key halves beyond every query of THIS wave (causal) or past Sk are
    // skipped by the wave (a wave-uniform branch); all waves still stage and sync
    int nlive = 2;
    if constexpr (MASK) {
      int kmax = Sk - 1;
      if (CAUSAL) kmax = min(kmax, q0 + wave * 32 + 31 + off);
      nlive = k0 > kmax ? 0 : (k0 + 32 > kmax ? 1 : 2);
      nlive = __builtin_amdgcn_readfirstlane(nlive);
    }
    if (nlive > 0) {
    // S^T = K Q^T : two 32-key tiles (raw scores). All 2*NS K fragments are read from LDS
    // before the first MFMA so the reads overlap each other instead of one LDS round trip
    // per MFMA (hipcc otherwise reuses one fragment register: read, wait, mfma, read, ...).
    f32x16 s_acc[2];
    {
      typename V8<T>::type kfr[2][NS];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int s = 0; s < NS; ++s)
          if (mt < nlive) kfr[mt][s] = frag_rows<T, D>(Ks, lo, mt, s);
      // nothing crosses this point: every read is issued before the first MFMA, and the
      // waitcnt pass then counts them down (lgkmcnt(N)) one MFMA at a time
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        if (mt < nlive) {
          s_acc[mt] = f32x16{};
#pragma unroll
          for (int s = 0; s < NS; ++s) s_acc[mt] = mfma<T>(kfr[mt][s], qf[s], s_acc[mt]);
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) s_acc[mt][i] = -INFINITY;
        }
      }
    }
    // V^T fragments of the PV product, issued right behind the S MFMAs (the K fragment
    // registers are free again) so the transposed LDS reads land under the softmax VALU
    // (the first two k-steps only: all four would exceed the 256-VGPR occupancy-2 budget)
    typename V8<T>::type vfr[2][ND];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) vfr[ks][dt] = frag_tr<T, D>(Vs, lo, dt, ks);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (MASK) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = k0 + 32 * mt + acc_row(i, h);
          const bool bad = key >= Sk || (CAUSAL && key > myq + off);
          s_acc[mt][i] = bad ? -INFINITY : s_acc[mt][i];
        }
    }
    if constexpr ((XF & XF_FMASK) != 0) {
      if (myq < Sq) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = k0 + 32 * mt + acc_row(i, h);
            if (mt < nlive && key < Sk) s_acc[mt][i] += fa_mask<T>(ext, b, hh, myq, key);
          }
      }
    } else if constexpr ((XF & XF_KMASK) != 0) {
      // element i <-> key k0 + 32mt + 8(i>>2) + 4h + (i&3): four float4 LDS reads per half
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 m4 = *reinterpret_cast<const float4*>(mrow + k0 + 32 * mt + 8 * g + 4 * h);
          s_acc[mt][4 * g + 0] += m4.x;
          s_acc[mt][4 * g + 1] += m4.y;
          s_acc[mt][4 * g + 2] += m4.z;
          s_acc[mt][4 * g + 3] += m4.w;
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s_acc[mt][i]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * scale_log2;
    const float m_new = fmaxf(m_run, mx);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    if (__any(m_new > m_run)) {  // exact: lanes whose max did not grow get alpha = 1
      const float alpha = fexp2(m_run - m_use);
      l_run *= alpha;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) acc_o[dt] *= alpha;
    }
    m_run = m_new;
    float ps = 0.f;
    uint32_t kbits[2] = {0u, 0u};  // this lane's keep bits of the two 32-key halves
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = fexp2(fmaf(s_acc[mt][i], scale_log2, -m_use));
        ps += p;  // the softmax denominator sums the undropped probabilities
        if constexpr ((XF & XF_DROP) != 0) {
          // elements i, i+1 (i even) are the adjacent keys of one hash pair. A dropped score
          // is zeroed here; the kept ones are scaled by 1/(1-p) once, in the output
          // normalisation. The keep bit goes to bit acc_row(i, 0) (constant); the lane half's
          // 4h offset is applied to the whole word below.
          const int kk = k0 + 32 * mt + acc_row(i & ~1, h);
          const uint32_t hs = fa_hash2(dkey, myq, kk >> 1);
          const bool keep = ((i & 1) ? (hs >> 16) : (hs & 0xffffu)) >= ext.thr;
          kbits[mt] |= keep ? (1u << acc_row(i, 0)) : 0u;
          p = keep ? p : 0.f;
        }
        s_acc[mt][i] = p;
      }
    if constexpr ((XF & XF_DROP) != 0) {
      if (ext.dbits) {  // both lane halves' 16 bits -> one word per (query, 32 keys)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const uint32_t kb = kbits[mt] << (4 * h);
          const uint32_t w = kb | __shfl_xor(kb, 32, 64);
          if (h == 0 && myq < Sq && mt < nlive)
            ext.dbits[((int64_t)bh * SqM + myq) * ext.dbits_ld + (k0 >> 5) + mt] = w;
        }
      }
    }
    ps += __shfl_xor(ps, 32, 64);
    l_run += ps;
    // O^T += V^T P^T (k-steps of a dead half contribute nothing)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks < 2 * nlive) {
        const typename V8<T>::type pf = pack_frag<T>(s_acc[ks >> 1], 8 * (ks & 1));
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
          acc_o[dt] = mfma<T>(ks < 2 ? vfr[ks & 1][dt] : frag_tr<T, D>(Vs, lo, dt, ks), pf, acc_o[dt]);
      }
    }
    }  // nlive > 0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile kt+1 landed
    __syncthreads();
  };
  // tiles [0, nfull) need no mask: every key < Sk and (causal) <= the block's first query
  int nfull = min(ntiles, Sk / kTile);
  if (CAUSAL) nfull = min(nfull, (q0 + off + 1) / kTile);
  if (nfull < 0) nfull = 0;
  auto run = [&](auto xf_c) __attribute__((always_inline)) {
    for (int kt = 0; kt < nfull; ++kt) tile(kt, std::false_type{}, xf_c);
    for (int kt = nfull; kt < ntiles; ++kt) tile(kt, std::true_type{}, xf_c);
  };
  if constexpr (!EXT) {
    run(std::integral_constant<int, 0>{});
  } else {
    switch (ext.xf) {
      case XF_DROP: run(std::integral_constant<int, XF_DROP>{}); break;
      case XF_KMASK: run(std::integral_constant<int, XF_KMASK>{}); break;
      case XF_KMASK | XF_DROP: run(std::integral_constant<int, XF_KMASK | XF_DROP>{}); break;
      case XF_FMASK: run(std::integral_constant<int, XF_FMASK>{}); break;
      case XF_FMASK | XF_DROP: run(std::integral_constant<int, XF_FMASK | XF_DROP>{}); break;
      default: run(std::integral_constant<int, 0>{}); break;
    }
  }

  if (myq < Sq) {
    float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    if constexpr (EXT) {
      if (ext.xf & XF_DROP) inv *= ext.inv_keep;  // the kept probabilities' 1/(1-p)
    }
    T* orow = o + (qrow0 + myq) * ((int64_t)H * D) + (int64_t)hh * D;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 w;
        w.x = pack2<T>(acc_o[dt][4 * g + 0] * inv, acc_o[dt][4 * g + 1] * inv);
        w.y = pack2<T>(acc_o[dt][4 * g + 2] * inv, acc_o[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d) = w;
      }
    if (h == 0) {
      const float l2 = l_run > 0.f ? (m_run + log2f(l_run)) : INFINITY;
      lse[(int64_t)bh * SqM + myq] = l2 * 0.6931471805599453f;
    }
  }
}

// ============================================================================
// backward: dQ (queries on lanes, sweep key tiles)
// ============================================================================
template <typename T, int D, bool CAUSAL, int NW>
__global__ void __launch_bounds__(NW * 64, 2)
bwd_dq_kernel(const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const T* __restrict__ dO,
              const T* __restrict__ o, const float* __restrict__ lse, float* __restrict__ delta, T* __restrict__ dq, int H, int Sq,
              int Sk, int64_t qsb, int64_t qss, int64_t qsh, int64_t ksb, int64_t kss, int64_t ksh, int64_t vsb,
              int64_t vss, int64_t vsh, int64_t dqsb, int64_t dqss, int64_t dqsh, float scale, float scale_log2) {
  // double-buffered {K, V} swizzled row images; K^T fragments by transposed reads of K
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* img0 = reinterpret_cast<T*>(smem);  // [2][2][64*D]
  constexpr int NS = D / 16, ND = D / 32, BM = NW * 32;
  const float LOG2E = 1.4426950408889634f;

  const int nqb = gridDim.y;
  const int qb = CAUSAL ? (nqb - 1 - blockIdx.y) : blockIdx.y;  // heaviest first (see fwd)
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int q0 = qb * BM;
  const int myq = q0 + wave * 32 + r;
  const int off = Sk - Sq;
  const bool qvalid = myq < Sq;

  const T* qb_ = q + b * qsb + hh * qsh;
  const T* kb_ = k + b * ksb + hh * ksh;
  const T* vb_ = v + b * vsb + hh * vsh;
  const int64_t HD = (int64_t)H * D;
  const T* dob_ = dO + (int64_t)b * Sq * HD + (int64_t)hh * D;

  typename V8<T>::type qf[NS], df[NS];
  {
    const int qq = qvalid ? myq : 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[s] = frag_global<T>(qb_ + (int64_t)qq * qss, 16 * s + 8 * h, qvalid);
      df[s] = frag_global<T>(dob_ + (int64_t)qq * HD, 16 * s + 8 * h, qvalid);
    }
  }
  const float lse2 = qvalid ? lse[(int64_t)bh * Sq + myq] * LOG2E : INFINITY;
  float dlt;
  if (o) {
    // delta = rowsum(dO * O) of this lane's query, computed here (the lane already holds its dO
    // row) and stored for the dK/dV kernel that runs next: no separate preprocess pass
    const T* ob_ = o + (int64_t)b * Sq * HD + (int64_t)hh * D;
    const int qq = qvalid ? myq : 0;
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const typename V8<T>::type of = frag_global<T>(ob_ + (int64_t)qq * HD, 16 * s + 8 * h, qvalid);
      const u32x4 uo = __builtin_bit_cast(u32x4, of), ud = __builtin_bit_cast(u32x4, df[s]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        part += lo16<T>(uo[j]) * lo16<T>(ud[j]) + hi16<T>(uo[j]) * hi16<T>(ud[j]);
    }
    dlt = part + __shfl_xor(part, 32, 64);
    if (qvalid && h == 0) delta[(int64_t)bh * Sq + myq] = dlt;
  } else {
    dlt = qvalid ? delta[(int64_t)bh * Sq + myq] : 0.f;
  }
  wait_vmem_all();

  f32x16 acc_q[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) acc_q[i] = f32x16{};

  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, q0 + BM + off);
  const int ntiles = n_end > 0 ? (n_end + kTile - 1) / kTile : 0;

  const LaneOffs<D> lo(lane);
  TileRegs<T, D, NW * 64> kr, vr;
  if (ntiles > 0) {
    kr.load(kb_, kss, 0, Sk);
    vr.load(vb_, vss, 0, Sk);
    kr.store_swz(img0);
    vr.store_swz(img0 + kTile * D);
  }
  __syncthreads();

  auto tile = [&](int kt, auto mask_c) {
    constexpr bool MASK = decltype(mask_c)::value;
    const int k0 = kt * kTile;
    const T* Ks = img0 + (2 * (kt & 1)) * kTile * D;
    const T* Vs = Ks + kTile * D;
    if (kt + 1 < ntiles) {
      kr.load(kb_, kss, k0 + kTile, Sk);
      vr.load(vb_, vss, k0 + kTile, Sk);
    }
    // masked tiles: 32-key halves past every query of THIS wave / past Sk are skipped
    int nlive = 2;
    if constexpr (MASK) {
      int kmax = Sk - 1;
      if (CAUSAL) kmax = min(kmax, q0 + wave * 32 + 31 + off);
      nlive = k0 > kmax ? 0 : (k0 + 32 > kmax ? 1 : 2);
      nlive = __builtin_amdgcn_readfirstlane(nlive);
    }
    if (nlive > 0) {
    f32x16 s_acc[2], dp_acc[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      s_acc[mt] = f32x16{};
      dp_acc[mt] = f32x16{};
      if (mt >= nlive) continue;
      // fragments read in groups of 2, one group ahead of the MFMAs that consume them
      // (this kernel is at the 256-VGPR occupancy-2 limit)
      constexpr int G = 2, NG = 2 * NS / G;  // groups over the K (first NS) then V fragments
      typename V8<T>::type fr[2][G];
#pragma unroll
      for (int g = 0; g <= NG; ++g) {
        if (g < NG) {
#pragma unroll
          for (int j = 0; j < G; ++j) {
            const int f = g * G + j;
            fr[g & 1][j] = f < NS ? frag_rows<T, D>(Ks, lo, mt, f) : frag_rows<T, D>(Vs, lo, mt, f - NS);
          }
        }
        if (g > 0) {
#pragma unroll
          for (int j = 0; j < G; ++j) {
            const int f = (g - 1) * G + j;
            if (f < NS) s_acc[mt] = mfma<T>(fr[(g - 1) & 1][j], qf[f], s_acc[mt]);
            else dp_acc[mt] = mfma<T>(fr[(g - 1) & 1][j], df[f - NS], dp_acc[mt]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = fexp2(fmaf(s_acc[mt][i], scale_log2, -lse2));
        if constexpr (MASK) {
          const int key = k0 + 32 * mt + acc_row(i, h);
          if (mt >= nlive || key >= Sk || (CAUSAL && key > myq + off)) p = 0.f;
        }
        s_acc[mt][i] = p * (dp_acc[mt][i] - dlt);  // dS^T (unscaled)
      }
    // dQ^T += K^T dS^T
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks < 2 * nlive) {
        const typename V8<T>::type sf = pack_frag<T>(s_acc[ks >> 1], 8 * (ks & 1));
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) acc_q[dt] = mfma<T>(frag_tr<T, D>(Ks, lo, dt, ks), sf, acc_q[dt]);
      }
    }
    }  // nlive > 0
    if (kt + 1 < ntiles) {  // idle buffer: last read before the previous barrier
      T* nb = img0 + (2 * ((kt + 1) & 1)) * kTile * D;
      kr.store_swz(nb);
      vr.store_swz(nb + kTile * D);
    }
    __syncthreads();
  };
  int nfull = min(ntiles, Sk / kTile);
  if (CAUSAL) nfull = min(nfull, (q0 + off + 1) / kTile);
  if (nfull < 0) nfull = 0;
  for (int kt = 0; kt < nfull; ++kt) tile(kt, std::false_type{});
  for (int kt = nfull; kt < ntiles; ++kt) tile(kt, std::true_type{});

  if (qvalid) {
    T* row = dq + (int64_t)b * dqsb + (int64_t)myq * dqss + (int64_t)hh * dqsh;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 w;
        w.x = pack2<T>(acc_q[dt][4 * g + 0] * scale, acc_q[dt][4 * g + 1] * scale);
        w.y = pack2<T>(acc_q[dt][4 * g + 2] * scale, acc_q[dt][4 * g + 3] * scale);
        *reinterpret_cast<uint2*>(row + d) = w;
      }
  }
}

// ============================================================================
// backward: dK, dV (keys on lanes, sweep query tiles)
// S = Q K^T with the 32x32 tile [q rows in registers, key = lane]:
//   A = Q (row-major LDS image), B = K^T (K fragments in registers)
// dV^T += dO^T P,  dK^T += Q^T dS  (A from transposed images, B = accumulators)
// ============================================================================
// WDS: also store dS^T (bf16/f16, unscaled) to dsT[bh][key][query] (row pitch Sqp, Skp rows) for
// bwd_dq_ds_kernel, which then forms dQ = dS K without recomputing S and dP.
// dK/dV kernel LDS: [2][Q | dO] tile images, lse / delta [2][64] each, the dS^T stage (NWV waves x
// 32 rows x 80 B), the keep-bit words (EXT), then the block's K / V images ([2][64][D] each)
template <typename T, int D, bool EXT, int NWV = 4>
__host__ __device__ constexpr int kKvOff() {
  return 4 * kTile * D * (int)sizeof(T) + 4 * kTile * 4 + NWV * 32 * 80 + (EXT ? 2 * 256 * 4 : 0);
}
template <typename T, int D, bool EXT, int NWV = 4>
__host__ __device__ constexpr int kDkdvLds() {
  return kKvOff<T, D, EXT, NWV>() + 4 * kTile * D * (int)sizeof(T);
}
// Query-split dK/dV (QS, head_dim 128): 8 waves per 128-key block, the pair (w, w + 4) sharing
// 32 keys and each taking one 32-query half of every tile, so a wave holds ONE half's S / dP
// accumulators (the dK / dV partials of its half) and the kernel runs two waves per SIMD: one
// wave's softmax VALU, LDS reads and barrier waits hide under its partner's MFMAs (at one wave
// per SIMD the dK/dV kernel measured ~25 % MFMA busy, profiles/r4/fa_pmc/summary.md). The pair's
// partials are summed through LDS once at the end.
__host__ __device__ constexpr int dkdv_waves(bool qs) { return qs ? 8 : 4; }

template <typename T, int D, bool CAUSAL, bool WDS, bool EXT = false, bool QS = false>
__global__ void __launch_bounds__(64 * dkdv_waves(QS), (D == 64 && !QS) ? 2 : 1)
bwd_dkdv_kernel(const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, const T* __restrict__ dO,
                const float* __restrict__ lse, const float* __restrict__ delta, T* __restrict__ dk,
                T* __restrict__ dv, int H, int SqM, int SkM, int64_t qsb, int64_t qss, int64_t qsh, int64_t ksb,
                int64_t kss, int64_t ksh, int64_t vsb, int64_t vss, int64_t vsh, int64_t dksb, int64_t dkss,
                int64_t dksh, int64_t dvsb, int64_t dvss, int64_t dvsh, float scale, float scale_log2,
                T* __restrict__ dsT, int Sqp, int64_t dsbh, FaExt ext = {}) {
  // Double-buffered LDS: buffer b = {Q image, dO image} (swizzled rows, read both row-wise and
  // transposed) + lse/delta of the tile's 64 queries. The next tile is written into the idle
  // buffer right after the current tile's MFMAs are issued: one barrier per tile.
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* img0 = reinterpret_cast<T*>(smem);                               // [2][2][64*D]
  float* Lsb = reinterpret_cast<float*>(img0 + 4 * kTile * D);        // [2][64] lse*log2e
  float* Dlb = Lsb + 2 * kTile;                                       // [2][64] delta
  constexpr int NS = D / 16, ND = D / 32;
  const float LOG2E = 1.4426950408889634f;

  constexpr int NWV = dkdv_waves(QS), NTH = 64 * NWV;
  const int kb = blockIdx.y;  // causal: key block 0 sweeps the most query tiles, launched first
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  // kw: the wave's 32-key group; qh (QS): the 32-query half of every tile it takes
  const int kw = QS ? (wave & 3) : wave, qh = QS ? (wave >> 2) : 0;
  const int kblk0 = kb * 128;
  const int mykey = kblk0 + kw * 32 + r;
  int Sq = SqM, Sk = SkM;
  int64_t qrow0 = (int64_t)b * SqM, krow0 = 0;
  if constexpr (EXT) {
    if (ext.cu_q) {
      qrow0 = ext.cu_q[b];
      krow0 = ext.cu_k[b];
      Sq = ext.cu_q[b + 1] - (int)qrow0;
      Sk = ext.cu_k[b + 1] - (int)krow0;
      if (kblk0 >= Sk) return;  // uniform, before any barrier
    }
  }
  const int off = Sk - Sq;
  const bool kvalid = mykey < Sk;
  const bool vl = EXT && ext.cu_q;

  const T* qb_ = vl ? q + qrow0 * qss + hh * qsh : q + b * qsb + hh * qsh;
  const T* kb_ = vl ? k + krow0 * kss + hh * ksh : k + b * ksb + hh * ksh;
  const T* vb_ = vl ? v + krow0 * vss + hh * vsh : v + b * vsb + hh * vsh;
  const int64_t HD = (int64_t)H * D;
  const T* dob_ = dO + qrow0 * HD + (int64_t)hh * D;

  // the block's 128 K and V rows live in LDS (two swizzled [64][D] images each, staged once by
  // LDS-DMA below; rows >= Sk read as zero) and each tile re-reads the wave's fragments: holding
  // them in registers for the whole kernel (64 VGPRs at D = 128) pushed the S / dP accumulators
  // into AGPRs, and every softmax element then paid v_accvgpr reads / writes
  const T* kvimg = reinterpret_cast<const T*>(smem + kKvOff<T, D, EXT, NWV>());
  const T* Kw = kvimg + (kw >> 1) * kTile * D;          // image holding this wave's 32 keys
  const T* Vw = kvimg + (2 + (kw >> 1)) * kTile * D;
  f32x16 acc_k[ND], acc_v[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) { acc_k[i] = f32x16{}; acc_v[i] = f32x16{}; }

  int q_begin = 0;
  if (CAUSAL) q_begin = max(0, kblk0 - off) / kTile * kTile;
  const int ntiles = q_begin < Sq ? (Sq - q_begin + kTile - 1) / kTile : 0;

  // Q / dO tiles by LDS-DMA straight into the swizzled images (rows >= Sq read as zero);
  // the tile's 64 lse / delta values go through registers
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  SwzDma<D, NTH> qd, dd;
  qd.init(qb_, qss, Sq, wave, lane);
  dd.init(dob_, HD, Sq, wave, lane);
  // EXT + dropout: the forward's keep-bit words of the tile's 64 queries x this block's 4 key
  // words ([2][4 waves][64] after the dS^T stage), staged with lse / delta
  const bool dbits = EXT && ext.thr && ext.dbits;
  uint32_t* Mb = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(Dlb + 2 * kTile) + NWV * 32 * 80);
  const uint32_t mb0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)Mb;
  const uint32_t lsb0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)Lsb;
  const uint32_t dlb0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)Dlb;
  // lse / delta / keep bits of the tile's 64 queries go to LDS by LDS-DMA too (rows >= Sq read 0;
  // the tail tile masks them): no register-staged loads in the loop, so no compiler-placed
  // vmcnt(0) ever waits for the Q / dO pieces just issued (it did: the loads' destination
  // registers are loop-carried, and the waitcnt pass drains everything before rewriting them)
  const u32x4 lse_rs = raw_desc(lse + (int64_t)bh * SqM, (uint64_t)Sq * 4);
  const u32x4 dl_rs = raw_desc(delta + (int64_t)bh * SqM, (uint64_t)Sq * 4);
  const u32x4 mb_rs = dbits ? raw_desc(ext.dbits + (int64_t)bh * SqM * ext.dbits_ld, (uint64_t)Sq * ext.dbits_ld * 4)
                            : u32x4{0u, 0u, 0u, 0u};
  auto load_tile = [&](int qs0) {
    const int nb = ((qs0 - q_begin) / kTile) & 1;
    const uint32_t img = lds0 + (uint32_t)((2 * nb) * kTile * D * sizeof(T));
    qd.issue(img, (uint32_t)((int64_t)qs0 * qss * 2), wave);
    dd.issue(img + kTile * D * sizeof(T), (uint32_t)((int64_t)qs0 * HD * 2), wave);
    if (wave == 0) dma_dword(lse_rs, (uint32_t)(qs0 + lane) * 4u, lsb0 + nb * kTile * 4);
    if (wave == 1) dma_dword(dl_rs, (uint32_t)(qs0 + lane) * 4u, dlb0 + nb * kTile * 4);
    if (dbits && wave < 4) {
      const int kwd = (kblk0 >> 5) + wave;
      const uint32_t off = kwd < ext.dbits_ld ? (uint32_t)(((int64_t)(qs0 + lane) * ext.dbits_ld + kwd) * 4) : 0x80000000u;
      dma_dword(mb_rs, off, mb0 + (nb * 256 + wave * 64) * 4);
    }
  };
  {
    SwzDma<D, NTH> kd2, vd2;
    kd2.init(kb_, kss, Sk, wave, lane);
    vd2.init(vb_, vss, Sk, wave, lane);
    const uint32_t kv0 = lds0 + (uint32_t)kKvOff<T, D, EXT, NWV>();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      kd2.issue(kv0 + (uint32_t)(j * kTile * D * sizeof(T)), (uint32_t)((int64_t)(kblk0 + 64 * j) * kss * 2), wave);
      vd2.issue(kv0 + (uint32_t)((2 + j) * kTile * D * sizeof(T)), (uint32_t)((int64_t)(kblk0 + 64 * j) * vss * 2),
                wave);
    }
  }
  if (ntiles > 0) load_tile(q_begin);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const LaneOffs<D> lo(lane);
  // dS^T of one 32-query half goes out through a wave-private [32 keys][32 queries] LDS stage
  // (80-B row pitch: conflict-free 8-B writes): lanes write their key row's packed fragments,
  // then read back 16 B each in row order, so the global stores are 64-B row segments (4 lanes
  // per key row) instead of 32 scattered 16-B pieces per store instruction.
  // Rows up to the 128-rounded Sk are allocated.
  constexpr int SP = 80;  // stage row pitch, bytes
  char* stage = reinterpret_cast<char*>(Dlb + 2 * kTile) + wave * 32 * SP;
  T* dsw = WDS ? dsT + (int64_t)bh * dsbh + (int64_t)(kblk0 + kw * 32 + (lane >> 2)) * Sqp + 8 * (lane & 3)
               : nullptr;
  // packed dS fragment of k-step ks (keys on lanes, queries 16ks + 4h + {0..3, 8..11} of the half)
  auto store_ds = [&](const typename V8<T>::type& sf, int ks) {
    const u32x4 u = __builtin_bit_cast(u32x4, sf);
    char* p = stage + r * SP + (16 * ks + 4 * h) * 2;
    *reinterpret_cast<u32x2*>(p) = u32x2{u[0], u[1]};
    *reinterpret_cast<u32x2*>(p + 16) = u32x2{u[2], u[3]};
  };
  // the half starting at query qh is complete in the stage: 2 x 16 rows x 64 B to dS^T
  auto flush_ds = [&](int qh) {
    const u32x4 a = *reinterpret_cast<const u32x4*>(stage + (lane >> 2) * SP + 16 * (lane & 3));
    const u32x4 c = *reinterpret_cast<const u32x4*>(stage + (16 + (lane >> 2)) * SP + 16 * (lane & 3));
    *reinterpret_cast<u32x4*>(dsw + qh) = a;
    *reinterpret_cast<u32x4*>(dsw + 16 * (int64_t)Sqp + qh) = c;
  };
  // XF_KMASK: the mask depends on the key only -> this lane's value, once
  float kmv = 0.f;
  if constexpr (EXT) {
    if ((ext.xf & XF_KMASK) && kvalid) {
      const int64_t i = (int64_t)b * ext.msb + (int64_t)hh * ext.msh + mykey;
      kmv = (ext.mask_f32 ? static_cast<const float*>(ext.mask)[i] : Cvt<T>::to(static_cast<const T*>(ext.mask)[i])) *
            ext.mask_mul;
    }
  }
  // XF (extended features of this copy of the loop): with XF_DROP the keep bits are always
  // the forward's stored ones (the launcher refuses dropout without them)
  auto tile = [&](int it, auto mask_c, auto xf_c) __attribute__((always_inline)) {
    constexpr bool MASK = decltype(mask_c)::value;
    constexpr int XF = decltype(xf_c)::value;
    const int buf = it & 1;
    const T* Qs = img0 + (2 * buf) * kTile * D;
    const T* Ds = Qs + kTile * D;
    const float* Ls = Lsb + buf * kTile;
    const float* Dl = Dlb + buf * kTile;
    const int qs0 = q_begin + it * kTile;
    if (it + 1 < ntiles) load_tile(qs0 + kTile);
    if constexpr (QS) {
      // one 32-query half (qh) of the tile: S^T / dP^T of the wave's 32 keys, softmax, then the
      // dV / dK updates; the k-step fragments are read as they are consumed (no fragment set
      // held across the tile: the wave stays within 256 registers)
      const int nt = qh;
      f32x16 sa = f32x16{}, da = f32x16{};
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2) {
        const typename V8<T>::type kf = frag_rows<T, D>(Kw, lo, kw & 1, s2);
        const typename V8<T>::type qf = frag_rows<T, D>(Qs, lo, nt, s2);
        const typename V8<T>::type vf = frag_rows<T, D>(Vw, lo, kw & 1, s2);
        const typename V8<T>::type df = frag_rows<T, D>(Ds, lo, nt, s2);
        sa = mfma<T>(qf, kf, sa);
        da = mfma<T>(df, vf, da);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *reinterpret_cast<const float4*>(Ls + 32 * nt + 8 * g + 4 * h);
        const float4 d4 = *reinterpret_cast<const float4*>(Dl + 32 * nt + 8 * g + 4 * h);
        const float la[4] = {l4.x * LOG2E, l4.y * LOG2E, l4.z * LOG2E, l4.w * LOG2E},
                    dl[4] = {d4.x, d4.y, d4.z, d4.w};
        uint4 mw = make_uint4(0u, 0u, 0u, 0u);
        if constexpr ((XF & XF_DROP) != 0)
          mw = *reinterpret_cast<const uint4*>(Mb + buf * 256 + kw * 64 + 32 * nt + 8 * g + 4 * h);
        const uint32_t mwa[4] = {mw.x, mw.y, mw.z, mw.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int i = 4 * g + c;
          const int qq = qs0 + 32 * nt + 8 * g + 4 * h + c;
          float sv = sa[i];
          if constexpr ((XF & XF_FMASK) != 0) {
            if (qq < Sq && kvalid) sv += fa_mask<T>(ext, b, hh, qq, mykey);
          } else if constexpr ((XF & XF_KMASK) != 0) {
            sv += kmv;
          }
          float p = fexp2(fmaf(sv, scale_log2, -la[c]));
          if constexpr (MASK) {
            if (qq >= Sq || (CAUSAL && mykey > qq + off)) p = 0.f;
          }
          if constexpr ((XF & XF_DROP) != 0) {
            const float z = (mwa[c] >> (mykey & 31)) & 1u ? ext.inv_keep : 0.f;
            sa[i] = p * z;
            da[i] = p * (da[i] * z - dl[c]);
            continue;
          }
          sa[i] = p;
          da[i] = p * (da[i] - dl[c]);
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const typename V8<T>::type pf = pack_frag<T>(sa, 8 * ks);
        const typename V8<T>::type sf = pack_frag<T>(da, 8 * ks);
        if constexpr (WDS) store_ds(sf, ks);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          const typename V8<T>::type dtr = frag_tr<T, D>(Ds, lo, dt, 2 * nt + ks);
          const typename V8<T>::type qtr = frag_tr<T, D>(Qs, lo, dt, 2 * nt + ks);
          acc_v[dt] = mfma<T>(dtr, pf, acc_v[dt]);
          acc_k[dt] = mfma<T>(qtr, sf, acc_k[dt]);
        }
      }
      if constexpr (WDS) flush_ds(qs0 + 32 * nt);
    } else {
      // software-pipelined tile: S/dP of BOTH 32-query halves first, then each half's softmax
      // VALU sits behind the other half's MFMAs in program order (nothing pins the order there),
      // so the matrix pipe keeps running while the exps issue. Masked tiles (causal diagonal,
      // Sq tail) run the same body with a per-element mask: a wave whose half is entirely
      // masked still computes it (P = dS = 0), which costs nothing on the tile's critical path
      // -- the barrier waits for the wave that has both halves live -- while the former
      // unpipelined masked body ran ~2.5x the VALU per tile on 20-25 % of the causal tiles.
      // dP starts from zero (MFMA with a zero C operand) and delta is subtracted in the softmax
      // VALU: seeding the accumulator with -delta cost a v_xor + a v_accvgpr_write per element
      // (the S/dP accumulators live in AGPRs at this register pressure)
      f32x16 sa[2], da[2];
      typename V8<T>::type kf[NS], vf[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        kf[s] = frag_rows<T, D>(Kw, lo, wave & 1, s);
        vf[s] = frag_rows<T, D>(Vw, lo, wave & 1, s);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        sa[nt] = f32x16{};
        da[nt] = f32x16{};
        typename V8<T>::type qfr[NS], dfr[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          qfr[s] = frag_rows<T, D>(Qs, lo, nt, s);
          dfr[s] = frag_rows<T, D>(Ds, lo, nt, s);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          sa[nt] = mfma<T>(qfr[s], kf[s], sa[nt]);
          da[nt] = mfma<T>(dfr[s], vf[s], da[nt]);
        }
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 l4 = *reinterpret_cast<const float4*>(Ls + 32 * nt + 8 * g + 4 * h);
          const float4 d4 = *reinterpret_cast<const float4*>(Dl + 32 * nt + 8 * g + 4 * h);
          const float la[4] = {l4.x * LOG2E, l4.y * LOG2E, l4.z * LOG2E, l4.w * LOG2E},
                      dl[4] = {d4.x, d4.y, d4.z, d4.w};
          uint4 mw = make_uint4(0u, 0u, 0u, 0u);
          if constexpr ((XF & XF_DROP) != 0)
            mw = *reinterpret_cast<const uint4*>(Mb + buf * 256 + kw * 64 + 32 * nt + 8 * g + 4 * h);
          const uint32_t mwa[4] = {mw.x, mw.y, mw.z, mw.w};
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int i = 4 * g + c;
            const int qq = qs0 + 32 * nt + 8 * g + 4 * h + c;
            float sv = sa[nt][i];
            if constexpr ((XF & XF_FMASK) != 0) {
              if (qq < Sq && kvalid) sv += fa_mask<T>(ext, b, hh, qq, mykey);
            } else if constexpr ((XF & XF_KMASK) != 0) {
              sv += kmv;
            }
            float p = fexp2(fmaf(sv, scale_log2, -la[c]));
            if constexpr (MASK) {
              if (qq >= Sq || (CAUSAL && mykey > qq + off)) p = 0.f;
            }
            if constexpr ((XF & XF_DROP) != 0) {
              // the forward's keep bit
              const float z = (mwa[c] >> (mykey & 31)) & 1u ? ext.inv_keep : 0.f;
              sa[nt][i] = p * z;
              da[nt][i] = p * (da[nt][i] * z - dl[c]);
              continue;
            }
            sa[nt][i] = p;
            da[nt][i] = p * (da[nt][i] - dl[c]);
          }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          typename V8<T>::type dtr[ND], qtr[ND];
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) {
            dtr[dt] = frag_tr<T, D>(Ds, lo, dt, 2 * nt + ks);
            qtr[dt] = frag_tr<T, D>(Qs, lo, dt, 2 * nt + ks);
          }
          const typename V8<T>::type pf = pack_frag<T>(sa[nt], 8 * ks);
          const typename V8<T>::type sf = pack_frag<T>(da[nt], 8 * ks);
          if constexpr (WDS) store_ds(sf, ks);
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) {
            acc_v[dt] = mfma<T>(dtr[dt], pf, acc_v[dt]);
            acc_k[dt] = mfma<T>(qtr[dt], sf, acc_k[dt]);
          }
        }
        if constexpr (WDS) flush_ds(qs0 + 32 * nt);
      }
    }
    // the idle buffer was last read before the previous barrier; its DMA (Q / dO / lse / delta /
    // keep bits) was issued at the top of this tile. Only the dS^T stores of this tile (WDS: 2 per
    // 32-query half, QS waves store one half) are younger: leave them in flight.
    if constexpr (WDS) wait_vm<QS ? 2 : 4>();
    else wait_vm<0>();
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS reads of the tile are done
    __builtin_amdgcn_s_barrier();
  };
  // query tiles that straddle the causal diagonal of this 128-key block (the first ones) or
  // Sq (the last one) need the mask; separate loops keep one body copy live at a time
  int it0 = 0;
  if (CAUSAL) {
    while (it0 < ntiles && kblk0 + 127 > q_begin + it0 * kTile + off) ++it0;
  }
  int it1 = ntiles;
  while (it1 > it0 && q_begin + (it1 - 1) * kTile + kTile > Sq) --it1;
  auto run = [&](auto xf_c) __attribute__((always_inline)) {
    for (int it = 0; it < it0; ++it) tile(it, std::true_type{}, xf_c);
    for (int it = it0; it < it1; ++it) tile(it, std::false_type{}, xf_c);
    for (int it = it1; it < ntiles; ++it) tile(it, std::true_type{}, xf_c);
  };
  if constexpr (!EXT) {
    run(std::integral_constant<int, 0>{});
  } else {
    switch (ext.xf) {
      case XF_DROP: run(std::integral_constant<int, XF_DROP>{}); break;
      case XF_KMASK: run(std::integral_constant<int, XF_KMASK>{}); break;
      case XF_KMASK | XF_DROP: run(std::integral_constant<int, XF_KMASK | XF_DROP>{}); break;
      case XF_FMASK: run(std::integral_constant<int, XF_FMASK>{}); break;
      case XF_FMASK | XF_DROP: run(std::integral_constant<int, XF_FMASK | XF_DROP>{}); break;
      default: run(std::integral_constant<int, 0>{}); break;
    }
  }

  if constexpr (QS) {
    // the pair's partial dK / dV (the two query halves) summed through LDS: the upper-half wave
    // parks its accumulators ([kw][register][lane] fp32, conflict-free), its partner adds them
    float* xa = reinterpret_cast<float*>(smem);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __syncthreads();  // every wave is done with the tile images and the dS^T stage
    if (qh == 1) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          xa[((kw * 2 * ND + dt) * 16 + e) * 64 + lane] = acc_k[dt][e];
          xa[((kw * 2 * ND + ND + dt) * 16 + e) * 64 + lane] = acc_v[dt][e];
        }
    }
    __syncthreads();
    if (qh == 0) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          acc_k[dt][e] += xa[((kw * 2 * ND + dt) * 16 + e) * 64 + lane];
          acc_v[dt][e] += xa[((kw * 2 * ND + ND + dt) * 16 + e) * 64 + lane];
        }
    }
    __syncthreads();  // the partial area is read before the stages below reuse it
  }
  // bias-gradient partials: this block's 128 rounded dK / dV rows go through two padded [128][D+4]
  // LDS stages (the tile images are free now), then thread t sums column t of [dK | dV]
  constexpr int RP = D + 4;
  T* sk = img0;
  T* sv = img0 + 128 * RP;
  const bool bs = ext.bsum != nullptr;  // uniform
  if (bs && !QS) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __syncthreads();  // every wave's reads of the last tile's images (and the dS^T stage) are done
  }
  const bool writer = !QS || qh == 0;   // QS: the lower-half wave of each pair holds the sums
  T* krow = (vl ? dk + krow0 * dkss : dk + (int64_t)b * dksb) + (int64_t)mykey * dkss + (int64_t)hh * dksh;
  T* vrow = (vl ? dv + krow0 * dvss : dv + (int64_t)b * dvsb) + (int64_t)mykey * dvss + (int64_t)hh * dvsh;
  const int srow = kw * 32 + r;
  if (writer)
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * h;
      uint2 wk, wv;
      wk.x = pack2<T>(acc_k[dt][4 * g + 0] * scale, acc_k[dt][4 * g + 1] * scale);
      wk.y = pack2<T>(acc_k[dt][4 * g + 2] * scale, acc_k[dt][4 * g + 3] * scale);
      wv.x = pack2<T>(acc_v[dt][4 * g + 0], acc_v[dt][4 * g + 1]);
      wv.y = pack2<T>(acc_v[dt][4 * g + 2], acc_v[dt][4 * g + 3]);
      if (kvalid) {
        *reinterpret_cast<uint2*>(krow + d) = wk;
        *reinterpret_cast<uint2*>(vrow + d) = wv;
      }
      if (bs) {
        const uint2 z = make_uint2(0u, 0u);
        *reinterpret_cast<uint2*>(sk + srow * RP + d) = kvalid ? wk : z;
        *reinterpret_cast<uint2*>(sv + srow * RP + d) = kvalid ? wv : z;
      }
    }
  if (bs) {
    __syncthreads();
    const int col = threadIdx.x;
    if (col < 2 * D) {
      const T* src = col < D ? sk + col : sv + (col - D);
      float a = 0.f;
#pragma unroll 8
      for (int i = 0; i < 128; ++i) a += Cvt<T>::to(src[i * RP]);
      const int64_t HD = (int64_t)H * D;
      ext.bsum[((int64_t)b * ext.bsum_nblk + kb) * 3 * HD + (col < D ? 1 : 2) * HD + (int64_t)hh * D + (col % D)] = a;
    }
  }
}

// ============================================================================
// backward: dQ = dS K from the dS^T the dK/dV kernel stored (queries on lanes, sweep key tiles).
// dQ^T += K^T dS^T: A = K^T and B = dS^T both by transposed reads of swizzled row images (K
// [64 keys][D], dS^T [64 keys][256 queries]) in the same permuted k order, so the operands
// agree key for key. dS^T entries above the causal diagonal were never written: masked here.
// 8 waves x 32 queries share one K tile; both images are filled by LDS-DMA
// (buffer_load ... lds: no VGPR staging, no ds_write) with per-lane source offsets that
// realise the swizzle, and the buffer range check zero-fills key rows >= Sk.
// ============================================================================
template <typename T, int D, bool CAUSAL, bool EXT = false, int NW = 8, int NBUF = 3>
__global__ void __launch_bounds__(NW * 64, 1)
bwd_dq_ds_kernel(const T* __restrict__ k, const T* __restrict__ dsT, T* __restrict__ dq, int H, int SqM, int SkM,
                 int Sqp, int64_t dsbh, int64_t ksb, int64_t kss, int64_t ksh, int64_t dqsb, int64_t dqss,
                 int64_t dqsh, float scale, FaExt ext = {}) {
  constexpr int NT = NW * 64, BM = NW * 32, ND = D / 32, BUF = kTile * D + kTile * BM;
  // NBUF-slot ring, tiles staged NBUF-1 ahead: the per-tile MFMA work (16 per wave) is far
  // shorter than a DMA round trip, so one tile in flight per CU left the kernel latency-bound
  static_assert(NBUF >= 2 && NBUF <= 4, "ring depth");
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  T* img0 = reinterpret_cast<T*>(smem);  // [NBUF][K image 64*D | dS^T image 64*BM]
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  const int nqb = gridDim.y;
  const int qb = CAUSAL ? (nqb - 1 - blockIdx.y) : blockIdx.y;  // heaviest first
  const int bh = blockIdx.x, b = bh / H, hh = bh % H;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int q0 = qb * BM;
  const int myq = q0 + wave * 32 + r;
  int Sq = SqM, Sk = SkM;
  int64_t qrow0 = 0, krow0 = 0;
  const bool vl = EXT && ext.cu_q;
  if constexpr (EXT) {
    if (ext.cu_q) {
      qrow0 = ext.cu_q[b];
      krow0 = ext.cu_k[b];
      Sq = ext.cu_q[b + 1] - (int)qrow0;
      Sk = ext.cu_k[b + 1] - (int)krow0;
      if (q0 >= Sq) return;  // uniform, before any barrier
    }
  }
  const int off = Sk - Sq;

  f32x16 acc_q[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) acc_q[i] = f32x16{};

  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, q0 + BM + off);
  const int ntiles = n_end > 0 ? (n_end + kTile - 1) / kTile : 0;

  const LaneOffs<D> lo(lane);
  const LaneOffs<BM> ls(lane);
  SwzDma<D, NT> kd;
  SwzDma<BM, NT> sd;
  kd.init(vl ? k + krow0 * kss + hh * ksh : k + b * ksb + hh * ksh, kss, Sk, wave, lane);
  sd.init(dsT + (int64_t)bh * dsbh + q0, Sqp, Sk, wave, lane);
  auto stage = [&](int kt) {
    const uint32_t img = lds0 + (uint32_t)((kt % NBUF) * BUF * sizeof(T));
    kd.issue(img, (uint32_t)((int64_t)kt * kTile * kss * 2), wave);
    sd.issue(img + kTile * D * sizeof(T), (uint32_t)((int64_t)kt * kTile * Sqp * 2), wave);
  };
  // DMA instructions per wave and stage: vmcnt(PER) leaves the newest stage in flight
  constexpr int PER = SwzDma<D, NT>::PER + SwzDma<BM, NT>::PER;
  static_assert(PER < 16, "vmcnt field");
  static_assert(PER * (NBUF - 1) < 64, "vmcnt field");
  // prologue: tiles 0 .. NBUF-2 staged; wait for tile 0 only
  int staged = 0;
  for (; staged < NBUF - 1 && staged < ntiles; ++staged) stage(staged);
  if (staged == NBUF - 1 && NBUF == 4) wait_vm<2 * PER>();
  else if (staged == NBUF - 1 && NBUF == 3) wait_vm<PER>();
  else if (staged == 2 && NBUF == 4) wait_vm<PER>();
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto tile = [&](int kt, auto mask_c) {
    constexpr bool MASK = decltype(mask_c)::value;
    const int k0 = kt * kTile;
    const T* Ks = img0 + (kt % NBUF) * BUF;
    const T* Ss = Ks + kTile * D;
    const bool ahead = kt + NBUF - 1 < ntiles;
    if (ahead) stage(kt + NBUF - 1);  // slot (kt+NBUF-1)%NBUF was last read in tile kt-1, before the last barrier
    int nlive = 2;
    if constexpr (MASK) {
      int kmax = Sk - 1;
      if (CAUSAL) kmax = min(kmax, q0 + wave * 32 + 31 + off);
      nlive = k0 > kmax ? 0 : (k0 + 32 > kmax ? 1 : 2);
      nlive = __builtin_amdgcn_readfirstlane(nlive);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks < 2 * nlive) {
        typename V8<T>::type bf = frag_tr<T, BM>(Ss, ls, wave, ks);
        if constexpr (MASK && CAUSAL) {
          // element j <-> key k0 + 16ks + 8(j>>2) + 4h + (j&3); keys past this query are zero
          u32x4 u = __builtin_bit_cast(u32x4, bf);
          const int kb0 = k0 + 16 * ks + 4 * h - off;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int key_lo = kb0 + 8 * (w >> 1) + 2 * (w & 1);
            const uint32_t mlo = key_lo > myq ? 0u : 0xffffu, mhi = key_lo + 1 > myq ? 0u : 0xffff0000u;
            u[w] &= (mlo | mhi);
          }
          bf = as_v8<T>(u);
        }
        typename V8<T>::type af[ND];
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) af[dt] = frag_tr<T, D>(Ks, lo, dt, ks);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) acc_q[dt] = mfma<T>(af[dt], bf, acc_q[dt]);
      }
    }
    // this wave's DMA of tile kt+1 landed (the younger stages may stay in flight)
    const int inflight = min(ntiles - 1 - (kt + 1), NBUF - 2);  // stages issued after tile kt+1's
    if (NBUF == 4 && inflight >= 2) wait_vm<2 * PER>();
    else if (inflight >= 1) wait_vm<PER>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  int nfull = min(ntiles, Sk / kTile);
  if (CAUSAL) nfull = min(nfull, (q0 + off + 1) / kTile);
  if (nfull < 0) nfull = 0;
  for (int kt = 0; kt < nfull; ++kt) tile(kt, std::false_type{});
  for (int kt = nfull; kt < ntiles; ++kt) tile(kt, std::true_type{});

  // bias-gradient partials (see FaExt::bsum): the block's BM rounded dQ rows through a padded
  // [BM][D+4] LDS stage, column sums per 128-row half
  constexpr int RP = D + 4;
  static_assert(BM * RP <= NBUF * BUF, "dQ stage fits the ring");
  T* sq = img0;
  const bool bs = ext.bsum != nullptr;  // uniform
  if (bs) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __syncthreads();
  }
  const bool qvalid = myq < Sq;
  T* row = (vl ? dq + qrow0 * dqss : dq + (int64_t)b * dqsb) + (int64_t)myq * dqss + (int64_t)hh * dqsh;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * h;
      uint2 w;
      w.x = pack2<T>(acc_q[dt][4 * g + 0] * scale, acc_q[dt][4 * g + 1] * scale);
      w.y = pack2<T>(acc_q[dt][4 * g + 2] * scale, acc_q[dt][4 * g + 3] * scale);
      if (qvalid) *reinterpret_cast<uint2*>(row + d) = w;
      if (bs) *reinterpret_cast<uint2*>(sq + (wave * 32 + r) * RP + d) = qvalid ? w : make_uint2(0u, 0u);
    }
  if (bs) {
    __syncthreads();
    for (int t = threadIdx.x; t < D * (BM / 128); t += NT) {
      const int half = t / D, col = t % D, blk = (q0 >> 7) + half;
      if (blk >= ext.bsum_nblk) continue;
      const T* src = sq + half * 128 * RP + col;
      float a = 0.f;
#pragma unroll 8
      for (int i = 0; i < 128; ++i) a += Cvt<T>::to(src[i * RP]);
      ext.bsum[((int64_t)b * ext.bsum_nblk + blk) * 3 * (int64_t)H * D + (int64_t)hh * D + col] = a;
    }
  }
}

template <typename T, int D, bool C, int NW>
static void launch_fwd_nw(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq,
                          int Sk, const int64_t* st, float scale, hipStream_t s) {
  const size_t lds = 4 * kTile * D * sizeof(T);
  auto kern = fwd_kernel<T, D, C, NW>;
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid(B * H, (Sq + NW * 32 - 1) / (NW * 32));
  hipLaunchKernelGGL(kern, grid, dim3(NW * 64), lds, s, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, H, Sq, Sk,
                     st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], st[8], scale * 1.4426950408889634f,
                     FaExt{});
}

// 8 waves = one 256-query block per CU (4-wave blocks, two per CU, measured the same)
template <typename T, int D, bool C>
static void launch_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq,
                       int Sk, const int64_t* st, float scale, hipStream_t s) {
  if (C) launch_fwd_nw<T, D, C, 4>(q, k, v, o, lse, B, H, Sq, Sk, st, scale, s);
  else launch_fwd_nw<T, D, C, 8>(q, k, v, o, lse, B, H, Sq, Sk, st, scale, s);
}

// dQ = dS K launch shape: waves per block x ring depth. PRA_FA_DQ_SHAPE = "8x3" (default: 256 queries
// per block, two tiles in flight), "8x2", "4x3", "4x4" (128 queries, three in flight) -- A/B knob.
static int dq_variant() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PRA_FA_DQ_SHAPE");
    v = 0;
    if (e && !strcmp(e, "8x2")) v = 1;
    else if (e && !strcmp(e, "4x3")) v = 2;
    else if (e && !strcmp(e, "4x4")) v = 3;
  }
  return v;
}

template <typename T, int D, bool C, bool EXT, int NW, int NBUF>
static void launch_dq_ds_cfg(const void* k, void* dsT, void* dq, int B, int H, int Sq, int Sk, int Sqp, int64_t dsbh,
                             const int64_t* st, float scale, const FaExt& ext, hipStream_t s) {
  const size_t lds = (size_t)NBUF * (kTile * D + kTile * NW * 32) * sizeof(T);
  auto kern = bwd_dq_ds_kernel<T, D, C, EXT, NW, NBUF>;
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(B * H, (Sq + NW * 32 - 1) / (NW * 32)), dim3(NW * 64), lds, s, (const T*)k,
                     (const T*)dsT, (T*)dq, H, Sq, Sk, Sqp, dsbh, st[3], st[4], st[5], st[9], st[10], st[11], scale,
                     ext);
}

template <typename T, int D, bool C, bool EXT>
static void launch_dq_ds(const void* k, void* dsT, void* dq, int B, int H, int Sq, int Sk, int Sqp, int64_t dsbh,
                         const int64_t* st, float scale, const FaExt& ext, hipStream_t s) {
  switch (dq_variant()) {
    case 1: launch_dq_ds_cfg<T, D, C, EXT, 8, 2>(k, dsT, dq, B, H, Sq, Sk, Sqp, dsbh, st, scale, ext, s); break;
    case 2: launch_dq_ds_cfg<T, D, C, EXT, 4, 3>(k, dsT, dq, B, H, Sq, Sk, Sqp, dsbh, st, scale, ext, s); break;
    case 3: launch_dq_ds_cfg<T, D, C, EXT, 4, 4>(k, dsT, dq, B, H, Sq, Sk, Sqp, dsbh, st, scale, ext, s); break;
    default: launch_dq_ds_cfg<T, D, C, EXT, 8, 3>(k, dsT, dq, B, H, Sq, Sk, Sqp, dsbh, st, scale, ext, s); break;
  }
}

// PRA_FA_DKDV_QS=0: head_dim 128 dK/dV on the 4-wave kernel (one wave per SIMD) instead of the
// query-split 8-wave one (A/B knob)
static bool dkdv_qs() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("PRA_FA_DKDV_QS");
    v = (e && !strcmp(e, "0")) ? 0 : 1;
  }
  return v == 1;
}

template <typename T, int D, bool C>
static void launch_bwd(const void* q, const void* k, const void* v, const void* dO, const void* o, const float* lse,
                       float* delta, void* dq, void* dk, void* dv, void* dsT, int B, int H, int Sq, int Sk,
                       const int64_t* st, float scale, float* bsum, hipStream_t s) {
  const float sl2 = scale * 1.4426950408889634f;
  if (dsT) {
    FaExt be{};
    be.bsum = bsum;
    be.bsum_nblk = (Sk + 127) / 128;
    // dK/dV first (stores dS^T), then dQ = dS K; `delta` is an input here
    const int Sqp = (Sq + 255) / 256 * 256;
    const int64_t dsbh = (int64_t)((Sk + 127) / 128 * 128) * Sqp;
    auto go = [&](auto qs_c) {
      constexpr bool QS = decltype(qs_c)::value;
      const size_t lds = kDkdvLds<T, D, false, dkdv_waves(QS)>();
      auto kern = bwd_dkdv_kernel<T, D, C, true, false, QS>;
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kern, dim3(B * H, (Sk + 127) / 128), dim3(64 * dkdv_waves(QS)), lds, s, (const T*)q,
                         (const T*)k, (const T*)v, (const T*)dO, lse, delta, (T*)dk, (T*)dv, H, Sq, Sk, st[0], st[1],
                         st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[12], st[13], st[14], st[15], st[16],
                         st[17], scale, sl2, (T*)dsT, Sqp, dsbh, be);
    };
    if (D == 128 && dkdv_qs()) go(std::true_type{});
    else go(std::false_type{});
    launch_dq_ds<T, D, C, false>(k, dsT, dq, B, H, Sq, Sk, Sqp, dsbh, st, scale, be, s);
    return;
  }
  {
    const size_t lds = 4 * kTile * D * sizeof(T);
    auto go = [&](auto nwc) {
      constexpr int NW = decltype(nwc)::value;
      auto kern = bwd_dq_kernel<T, D, C, NW>;
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(kern, dim3(B * H, (Sq + NW * 32 - 1) / (NW * 32)), dim3(NW * 64), lds, s, (const T*)q,
                         (const T*)k, (const T*)v, (const T*)dO, (const T*)o, lse, delta, (T*)dq, H, Sq, Sk, st[0], st[1], st[2],
                         st[3], st[4], st[5], st[6], st[7], st[8], st[9], st[10], st[11], scale, sl2);
    };
    go(std::integral_constant<int, 8>{});
  }
  auto go = [&](auto qs_c) {
    constexpr bool QS = decltype(qs_c)::value;
    const size_t lds = kDkdvLds<T, D, false, dkdv_waves(QS)>();
    auto kern = bwd_dkdv_kernel<T, D, C, false, false, QS>;
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(B * H, (Sk + 127) / 128), dim3(64 * dkdv_waves(QS)), lds, s, (const T*)q,
                       (const T*)k, (const T*)v, (const T*)dO, lse, delta, (T*)dk, (T*)dv, H, Sq, Sk, st[0], st[1],
                       st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[12], st[13], st[14], st[15], st[16],
                       st[17], scale, sl2, (T*)nullptr, 0, (int64_t)0, FaExt{});
  };
  // (the same dK/dV kernel as the dS^T path: dV is bit-identical between the two dQ paths)
  if (D == 128 && dkdv_qs()) go(std::true_type{});
  else go(std::false_type{});
}

// extended variants (varlen / additive mask / dropout): forward + the dS^T backward
template <typename T, int D, bool C>
static void launch_fwd_ext(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq,
                           int Sk, const int64_t* st, float scale, const FaExt& ext, hipStream_t s) {
  constexpr int NW = C ? 4 : 8;
  size_t lds = 4 * kTile * D * sizeof(T);
  if (ext.xf & XF_KMASK) lds += (size_t)((Sk + kTile - 1) / kTile * kTile) * sizeof(float);  // mask row
  auto kern = fwd_kernel<T, D, C, NW, true>;
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid(B * H, (Sq + NW * 32 - 1) / (NW * 32));
  hipLaunchKernelGGL(kern, grid, dim3(NW * 64), lds, s, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, H, Sq, Sk,
                     st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], st[8], scale * 1.4426950408889634f, ext);
}

template <typename T, int D, bool C>
static void launch_bwd_ext(const void* q, const void* k, const void* v, const void* dO, const float* lse,
                           const float* delta, void* dq, void* dk, void* dv, void* dsT, int B, int H, int Sq, int Sk,
                           const int64_t* st, float scale, const FaExt& ext, hipStream_t s) {
  const float sl2 = scale * 1.4426950408889634f;
  const int Sqp = (Sq + 255) / 256 * 256;
  const int64_t dsbh = (int64_t)((Sk + 127) / 128 * 128) * Sqp;
  auto go = [&](auto qs_c) {
    constexpr bool QS = decltype(qs_c)::value;
    const size_t lds = kDkdvLds<T, D, true, dkdv_waves(QS)>();
    auto kern = bwd_dkdv_kernel<T, D, C, true, true, QS>;
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3(B * H, (Sk + 127) / 128), dim3(64 * dkdv_waves(QS)), lds, s, (const T*)q,
                       (const T*)k, (const T*)v, (const T*)dO, lse, delta, (T*)dk, (T*)dv, H, Sq, Sk, st[0], st[1],
                       st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[12], st[13], st[14], st[15], st[16],
                       st[17], scale, sl2, (T*)dsT, Sqp, dsbh, ext);
  };
  if (D == 128 && dkdv_qs()) go(std::true_type{});
  else go(std::false_type{});
  launch_dq_ds<T, D, C, true>(k, dsT, dq, B, H, Sq, Sk, Sqp, dsbh, st, scale, ext, s);
}

}  // namespace fa
}  // namespace pra

using namespace pra;

#define PRA_FA_DISPATCH(FN, ...)                                                                  \
  do {                                                                                             \
    if (dt == kBF16) {                                                                             \
      if (D == 128) { if (causal) fa::FN<bf16, 128, true>(__VA_ARGS__); else fa::FN<bf16, 128, false>(__VA_ARGS__); } \
      else { if (causal) fa::FN<bf16, 64, true>(__VA_ARGS__); else fa::FN<bf16, 64, false>(__VA_ARGS__); } \
    } else {                                                                                       \
      if (D == 128) { if (causal) fa::FN<f16, 128, true>(__VA_ARGS__); else fa::FN<f16, 128, false>(__VA_ARGS__); } \
      else { if (causal) fa::FN<f16, 64, true>(__VA_ARGS__); else fa::FN<f16, 64, false>(__VA_ARGS__); } \
    }                                                                                              \
  } while (0)

// FaExt of one extended launch: dropout threshold on 16-bit uniforms, the feature set (XF_*)
static fa::FaExt fa_ext(const int* cu_q, const int* cu_k, const void* mask, int64_t msb, int64_t msh, int64_t msq,
                        int mask_f32, float scale, float p_drop, uint64_t seed, uint64_t offset, uint32_t* dbits,
                        int Sk, const uint64_t* dseq) {
  uint32_t thr = (uint32_t)std::min<long long>(65535, std::llround((double)p_drop * 65536.0));
  int xf = 0;
  if (thr > 0) xf |= fa::XF_DROP;
  if (mask) xf |= (msq == 0 && Sk <= 4096) ? fa::XF_KMASK : fa::XF_FMASK;
  return fa::FaExt{cu_q, cu_k, mask, msb, msh, msq, mask_f32, 1.f / scale, thr,
                   thr > 0 ? (float)(65536.0 / (65536.0 - thr)) : 1.f, seed, offset, dbits, (Sk + 31) / 32, xf,
                   dseq};
}

extern "C" {
int pra_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq, int Sk,
                  int D, const int64_t* strides, float scale, int causal, int dt, hipStream_t s) {
  if (!(D == 64 || D == 128) || !(dt == kBF16 || dt == kF16)) return -1;
  if (B * H == 0 || Sq == 0) return 0;
  PRA_FA_DISPATCH(launch_fwd, q, k, v, o, lse, B, H, Sq, Sk, strides, scale, s);
  return 0;
}
// o != nullptr: delta = rowsum(dO * O) is computed inside the dQ kernel (o and dO [B, Sq, H, D]
// contiguous) and written to `delta` for the dK/dV kernel; o == nullptr: `delta` is an input.
// dsT != nullptr (requires o == nullptr): dS^T scratch of B*H*roundup(Sk,128)*roundup(Sq,256)
// elements; dQ = dS K is formed from it instead of recomputing S and dP in a dQ sweep.
// Extended forward: varlen (cu_q / cu_k [B+1] row prefix sums of packed [total, H, D] q/k/v/o;
// Sq, Sk = the longest sequences; lse [B, H, Sq]), additive mask (element strides msb / msh /
// msq, keys contiguous; mask_f32: fp32 else q's dtype), dropout p_drop with (seed, offset);
// dbits (optional, B*H*Sq*ceil(Sk/32) words) receives the keep bits for the backward.
int pra_flash_fwd_ext(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq, int Sk,
                      int D, const int64_t* strides, float scale, int causal, int dt, const int* cu_q,
                      const int* cu_k, const void* mask, int64_t msb, int64_t msh, int64_t msq, int mask_f32,
                      float p_drop, uint64_t seed, uint64_t offset, uint32_t* dbits, const uint64_t* dseq,
                      hipStream_t s) {
  if (!(D == 64 || D == 128) || !(dt == kBF16 || dt == kF16)) return -1;
  if (!(p_drop >= 0.f && p_drop < 1.f) || (!cu_q) != (!cu_k)) return -1;
  if (B * H == 0 || Sq == 0) return 0;
  const fa::FaExt e = fa_ext(cu_q, cu_k, mask, msb, msh, msq, mask_f32, scale, p_drop, seed, offset, dbits, Sk, dseq);
  PRA_FA_DISPATCH(launch_fwd_ext, q, k, v, o, lse, B, H, Sq, Sk, strides, scale, e, s);
  return 0;
}
// Extended backward (same extras as the forward; `delta` = rowsum(dO*O) [B, H, Sq] is an input,
// dsT the dS^T scratch of B*H*roundup(Sk,128)*roundup(Sq,256) elements). bsum (optional, both
// backward entries): [B * ceil(S/128)][3*H*D] fp32 column-sum partials of the packed dQKV, the
// bias gradient of the QKV projection before its row reduction (FaExt::bsum).
int pra_flash_bwd_ext(const void* q, const void* k, const void* v, const void* dO, const float* lse,
                      const float* delta, void* dq, void* dk, void* dv, void* dsT, int B, int H, int Sq, int Sk, int D,
                      const int64_t* strides, float scale, int causal, int dt, const int* cu_q, const int* cu_k,
                      const void* mask, int64_t msb, int64_t msh, int64_t msq, int mask_f32, float p_drop,
                      uint64_t seed, uint64_t offset, uint32_t* dbits, const uint64_t* dseq, float* bsum,
                      hipStream_t s) {
  if (!(D == 64 || D == 128) || !(dt == kBF16 || dt == kF16) || !dsT) return -1;
  if (!(p_drop >= 0.f && p_drop < 1.f) || (!cu_q) != (!cu_k)) return -1;
  if (bsum && (cu_q || Sq != Sk)) return -4;  // bias partials: packed self-attention only
  if (B * H == 0 || Sq == 0) return 0;
  fa::FaExt e = fa_ext(cu_q, cu_k, mask, msb, msh, msq, mask_f32, scale, p_drop, seed, offset, dbits, Sk, dseq);
  e.bsum = bsum;
  e.bsum_nblk = (Sk + 127) / 128;
  if ((e.xf & fa::XF_DROP) && !dbits) return -3;  // the backward reads the forward's keep bits
  PRA_FA_DISPATCH(launch_bwd_ext, q, k, v, dO, lse, delta, dq, dk, dv, dsT, B, H, Sq, Sk, strides, scale, e, s);
  return 0;
}
int pra_flash_bwd(const void* q, const void* k, const void* v, const void* dO, const void* o, const float* lse,
                  float* delta, void* dq, void* dk, void* dv, void* dsT, int B, int H, int Sq, int Sk, int D,
                  const int64_t* strides, float scale, int causal, int dt, float* bsum, hipStream_t s) {
  if (!(D == 64 || D == 128) || !(dt == kBF16 || dt == kF16)) return -1;
  if (dsT && o) return -2;
  if (bsum && (!dsT || Sq != Sk)) return -4;  // bias partials: the dS^T path, self-attention
  if (B * H == 0 || Sq == 0) return 0;
  PRA_FA_DISPATCH(launch_bwd, q, k, v, dO, o, lse, delta, dq, dk, dv, dsT, B, H, Sq, Sk, strides, scale, bsum, s);
  return 0;
}
}
