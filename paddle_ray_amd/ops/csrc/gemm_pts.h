// Persistent TS GEMM (PTS): one 256x256-tile workgroup per CU walks its tiles back to back.
//
// Why: on the GPT shapes the per-tile overhead of the one-launch-per-tile kernel (gemm_lds_kernel)
// is ~20k shader cycles -- a 5-8k-cycle DMA prologue, a 10-13k-cycle LDS-staged epilogue and a
// ~1.3k-cycle launch gap (profiles/r4/gemm_stamps_*.log) -- 20-25 % of a K=2048 tile's K loop.
// hipBLASLt's gfx950 kernels are persistent (profiles/r4/pmc_fc1_dgrad: 256 workgroups, 2 tiles
// each). Here the K-step stream simply continues across tiles:
//   * the K loop is the TS schedule of gemm_core.h (kstep_t): a K-step's fragments are read in its
//     first MFMAs, the refill of step kt+2 is spread one piece per 5 (W4) / 4 (W8) MFMAs, the
//     counted vmcnt comes late;
//   * in a tile's last two K-steps the refill pieces are the NEXT tile's steps 0 and 1 (slot =
//     step parity, K/64 even), so the next tile starts computing right after the epilogue, its
//     operands already in LDS (its first fragments are read after the epilogue: registers);
//   * the epilogue never touches the two LDS slots (they hold the next tile's steps): bias /
//     activation / dGELU / beta run on the accumulators in registers, v_permlane16_swap pairs the
//     4-column pieces of adjacent 16-column blocks so every lane stores 8 consecutive outputs
//     (16-B stores, 64 B per row per instruction); the dGELU column sums (bias gradient) reduce
//     across lanes by shuffles and across the two wave rows through a 1-KB LDS area beside the
//     slots, one partial row per tile ([tiles_m][N], as gemm_lds_kernel);
//   * the first K-step of a tile runs its first-half MFMAs with a zero accumulator input (no
//     accumulator clearing pass).
// Tile order: workgroup b serves tiles w, w + G, w + 2G, ... with w the XCD-major rank of b, so the
// workgroups of one XCD always work on a contiguous run of the 8-row-grouped tile order (L2 reuse).
// Requirements (checked by the host entry): K % 128 == 0 and K >= 256, bf16/f16, no split-K.
#pragma once
#include "gemm_core.h"

namespace pra {
namespace {

template <typename T>
__device__ __forceinline__ void mma_agpr_z(typename V8<T>::type a, typename V8<T>::type b, f32x4& c);
template <>
__device__ __forceinline__ void mma_agpr_z<bf16>(V8<bf16>::type a, V8<bf16>::type b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}
template <>
__device__ __forceinline__ void mma_agpr_z<f16>(V8<f16>::type a, V8<f16>::type b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}

// inclusive scan over the 16 lanes of a DPP row: lane 15 of each row returns the row's sum
__device__ __forceinline__ float row16_sum(float x) {
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x111, 0xf, 0xf, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x112, 0xf, 0xf, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x114, 0xf, 0xf, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x118, 0xf, 0xf, true));
  return x;
}

// VAR (measurement variants): bits 0-7 = MFMA slots between two refill pieces of a K-step (0:
// spread them over the whole window between the two barriers); bit 8 = read the next step's
// first A fragment ahead of the B fragments (every first-use gets the same MFMA slack); bits
// 12-15 = move the second barrier this many MFMA slots earlier.
// dynamic-order counters: one per XCD, each in its own 256-B line
constexpr int kPtsCtrStride = 64;

template <typename T, typename CF, bool AK, bool BK, int E, bool BETA, int VAR = 0>
__global__ __launch_bounds__(CF::NT, 1) void gemm_pts_kernel(const uint16_t* __restrict__ A,
                                                             const uint16_t* __restrict__ B,
                                                             const uint16_t* __restrict__ bias,
                                                             uint16_t* __restrict__ C, uint16_t* __restrict__ Z,
                                                             float* __restrict__ colsum, int M, int N, int K, int lda,
                                                             int ldb, int ldc, int ldz, int* __restrict__ tctr,
                                                             int nts) {
  constexpr int NT = CF::NT, TI = CF::TI, TJ = CF::TJ, NDA = CF::NDA, NDB = CF::NDB, WC = CF::WC;
  constexpr int BM = CF::BM, BN = CF::BN, IMGA = CF::IMGA, SLOT = CF::SLOT;
  constexpr int RW = TI * 16, CW = TJ * 16;
  constexpr bool AGPR_ACC = CF::WR * CF::WC == 4;
  static_assert(BM == 256 && BN == 256 && TJ % 2 == 0 && CF::WR == 2, "pts: 256x256 tiles, 2 wave rows");
  __shared__ __attribute__((aligned(1024))) char lds[2 * SLOT + 2 * BN * 4 + 16];
  typedef typename V8<T>::type v8;
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN, ntiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  // XCD-major rank of this workgroup (bijective for any G): the workgroups of XCD x own the
  // ranks [x0, x0 + nx); round k of the static order gives them tiles k * G + [x0, x0 + nx)
  const int xq = G >> 3, xr = G & 7, xcd = blockIdx.x & 7;
  const int nx = xcd < xr ? xq + 1 : xq, x0 = xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq;
  int pid = x0 + (blockIdx.x >> 3);
  if (pid >= ntiles) return;
  // tctr (dynamic order): the same per-XCD tile runs, but which workgroup of the XCD takes the
  // next one is decided by a per-XCD counter (one vector atomic per tile, fetched a K-step
  // ahead): a workgroup slowed by a co-resident kernel (RCCL channels during overlapped
  // communication) takes fewer tiles instead of stretching the whole GEMM
  int* nxt_lds = reinterpret_cast<int*>(lds + 2 * SLOT + 2 * BN * 4);
  // tiles of this XCD's runs (ranks r with (r / nx) * G + x0 + r % nx < ntiles: a prefix)
  const int tx = (ntiles / G) * nx + min(max(ntiles % G - x0, 0), nx);
  auto tile_mn = [&](int p, int& tm, int& tn) {
    const int group = 8 * tiles_n, gi = p / group, first_m = gi * 8;
    const int gm = min(tiles_m - first_m, 8);
    tm = first_m + (p % group) % gm;
    tn = (p % group) / gm;
  };
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), wr = wave / WC,
            wc = wave % WC;

  typedef Dma<AK, NT, NDA, CF::BUF, (AK ? 256 : BM), CF::SC1> DmaA;
  typedef Dma<BK, NT, NDB, CF::BUF, 256, CF::SC1> DmaB;
  DmaA da;
  DmaB db;
  auto dma_init = [&](DmaA& xa, DmaB& xb, int tm, int tn) {
    const int m0 = tm * BM, n0 = tn * BN;
    if (AK) xa.init(A, lda, m0, M - 1, tid);
    else xa.init(A, lda, m0, M - 8, tid);
    if (BK) xb.init(B, ldb, n0, N - 1, tid);
    else xb.init(B, ldb, n0, N - 8, tid);
  };
  const int nk = K / BKT;  // even, >= 4

  f32x4 acc[TI][TJ];
  v8 fa0[TI], fb0[TJ], fa1[TI], fb1[TJ];

  int tm, tn;
  tile_mn(pid, tm, tn);
  dma_init(da, db, tm, tn);
  // prologue of the first tile: steps 0 and 1 in flight, step 0's first fragments in registers
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int n = 0; n < NDA; ++n) da.issue1(lds_base + t * SLOT, wave, t, n);
#pragma unroll
    for (int n = 0; n < NDB; ++n) db.issue1(lds_base + t * SLOT + IMGA, wave, t, n);
  }
  wait_vmcnt<NDA + NDB>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  {
    const char* ai = lds;
    const char* bi = ai + IMGA;
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb0[j] = frag<T, BK>(bi, wc * CW + j * 16, 0, lane);
#pragma unroll
    for (int i = 0; i < TI; ++i) fa0[i] = frag<T, AK, (AK ? 256 : BM)>(ai, wr * RW + i * 16, 0, lane);
  }

  // The epilogue's Z (scaling epilogues) / C (beta) operand of the current tile: loaded into
  // registers in the last K-step, in the MFMA slots after its final barrier (the fragment
  // registers of the next K-step are free there: the next tile's first fragments are read after
  // the epilogue), so the loads' latency and bandwidth overlap the last 16-18 MFMAs instead of
  // stalling a serialised epilogue (measured at 16384 x 8192 x 2048: reading Z inside the
  // epilogue cost ~100 us over the plain GEMM, beta=1 ~60 us).
  // Rows are streamed through a 3-deep register ring (16-row block i + 2 loads while block i is
  // processed; blocks 0 and 1 come from the K loop): the whole tile at once (128 VGPRs) spilled.
  constexpr bool ZOP = epi_scales(E) || BETA;
  constexpr bool DG = epi_scales(E);
  constexpr int NH = DG ? TJ / 2 : 1, JH = TJ / NH;  // epilogue column passes (one block pair each), blocks per pass
  constexpr int ZR = 3;                          // ring depth (pass-rows in flight)
  uint2 gza[ZOP ? ZR : 1][ZOP ? JH : 1];
  const uint16_t* zp = nullptr;
  int zr0 = 0, zc0 = 0, zld = 0;
  // element l = q * JH + jq of pass-row q = hp * TI + i (16-row block i, column pass hp)
  auto zload = [&](int l) __attribute__((always_inline)) {
    if constexpr (ZOP) {
      const int q = l / JH, jq = l % JH, hp = q / TI, i = q % TI, j = hp * JH + jq;
      if (q < NH * TI) {
        gza[q % ZR][jq] = make_uint2(0u, 0u);
        if (zr0 + i * 16 < M && zc0 + j * 16 < N)
          gza[q % ZR][jq] = *reinterpret_cast<const uint2*>(zp + (int64_t)(i * 16) * zld + j * 16);
      }
    }
  };

  // one TS K-step (see gemm_core.h kstep_t); FIRST: the half-0 MFMAs start from a zero
  // accumulator. Outside STEADY the refill target (this tile's step kt+2, the next tile's step
  // kt+2-nk, or none) and the next-fragment reads are runtime choices. ZPRE: issue the epilogue
  // operand loads (zload) after the final barrier (the tile's last K-step).
  auto kstep = [&](int kt, auto steady_c, auto first_c, bool dcur, bool dnext, bool rd1, auto zpre_c)
      __attribute__((always_inline)) {
    constexpr bool STEADY = decltype(steady_c)::value, FIRST = decltype(first_c)::value;
    constexpr bool ZPRE = decltype(zpre_c)::value && ZOP;
    constexpr int NRD = TI + TJ, NDMA = NDA + NDB, NM = TI * TJ, F = 2 * NM;
    constexpr int SPO = VAR & 255, BSH = (VAR >> 12) & 15;
    constexpr bool AFIRST = (VAR >> 8) & 1;
    constexpr int BA = NRD + 4, BB = F - NRD - 3 - BSH;
    constexpr int SP0 = (BB - BA - 1) / NDMA > 0 ? (BB - BA - 1) / NDMA : 1;
    constexpr int SP = SPO > 0 ? SPO : SP0;
    static_assert(BB >= NM && BA + 1 + (NDMA - 1) * SP < BB, "pts: fillers exceed the K-step's MFMAs");
    if constexpr (STEADY) {
      dcur = true;
      dnext = false;
      rd1 = true;
    }
    const bool dma = dcur || dnext;
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
            if constexpr (FIRST) {
              if constexpr (AGPR_ACC) mma_agpr_z<T>(fb0[j], fa0[i], acc[i][j]);
              else acc[i][j] = mma<T>(fb0[j], fa0[i], f32x4{0.f, 0.f, 0.f, 0.f});
            } else {
              if constexpr (AGPR_ACC) mma_agpr<T>(fb0[j], fa0[i], acc[i][j]);
              else acc[i][j] = mma<T>(fb0[j], fa0[i], acc[i][j]);
            }
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
              // (dnext: da / db already describe the next tile)
              const int st = dnext ? kt + 2 - nk : kt + 2;
              if (d < NDA) da.issue1(soA, wave, st, d);
              else db.issue1(soB, wave, st, d - NDA);
            }
          } else if (f == BB) {
            if (dma) wait_vmcnt<NDMA>();  // step kt+1's pieces landed (the refill still in flight)
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // ... for every wave
          } else if (rd1 && f > BB && f - BB - 1 < NRD) {
            const int r = f - BB - 1;
            if constexpr (AFIRST) {
              // A0, B0..B(TJ-1), A1.. : the first MFMA's operands are the first two reads
              if (r == 0) fa0[0] = frag<T, AK, (AK ? 256 : BM)>(an, wr * RW, 0, lane);
              else if (r <= TJ) fb0[r - 1] = frag<T, BK>(bn, wc * CW + (r - 1) * 16, 0, lane);
              else fa0[r - TJ] = frag<T, AK, (AK ? 256 : BM)>(an, wr * RW + (r - TJ) * 16, 0, lane);
            } else {
              if (r < TJ) fb0[r] = frag<T, BK>(bn, wc * CW + r * 16, 0, lane);
              else fa0[r - TJ] = frag<T, AK, (AK ? 256 : BM)>(an, wr * RW + (r - TJ) * 16, 0, lane);
            }
          } else if (ZPRE && f > BB) {
            // the ring's first ZR - 1 pass-rows, spread over the slots after the barrier
            constexpr int LPS = ((ZR - 1) * JH + (F - BB - 2)) / (F - BB - 1);  // loads per slot
#pragma unroll
            for (int q = 0; q < LPS; ++q)
              if ((f - BB - 1) * LPS + q < (ZR - 1) * JH) zload((f - BB - 1) * LPS + q);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
    if constexpr (!STEADY) __builtin_amdgcn_s_waitcnt(0xC07F);
  };

  float* xlds = reinterpret_cast<float*>(lds + 2 * SLOT);  // [2][BN] column sums per wave row
  while (true) {
    // the counter atomic is a plain (compiler-tracked) vector atomic: its result is consumed
    // after step 0, where the compiler's vmcnt(0) for it also retires step 2's refills a little
    // early. (An inline-asm atomic whose result the waitcnt model cannot see was spilled to
    // scratch before it returned by the register-heavy xᵀ·dy instantiations.)
    int fetched = 0;
    if (tctr && wave == 0 && lane == 0) fetched = atomicAdd(tctr + xcd * kPtsCtrStride, 1);
    int ntm = 0, ntn = 0;
    kstep(0, std::true_type{}, std::true_type{}, true, false, true, std::false_type{});
    if (tctr && wave == 0 && lane == 0) {
      const int f = nx + fetched;
      nxt_lds[0] = (f / nx) * G + x0 + f % nx;
      // the XCD's last fetch (its workgroups fetch once per tile they run: tx in all) returns the
      // counter to zero for the next launch on this stream; no workgroup fetches after it
      if (fetched == tx - 1) atomicExch(tctr + xcd * kPtsCtrStride, 0);
    }
    for (int kt = 1; kt + 2 < nk; ++kt)
      kstep(kt, std::true_type{}, std::false_type{}, true, false, true, std::false_type{});
    // (the LDS slot was written before step 1's barriers and is rewritten only after the next
    // tile's step 0, two barriers after every wave read it here)
    const int npid = tctr ? __builtin_amdgcn_readfirstlane(nxt_lds[0]) : pid + G;
    const bool has_next = (unsigned)npid < (unsigned)ntiles;  // (a bad dynamic fetch exits instead of faulting)
    // this tile's last refill was step nk-1 (issued in step nk-3): the DMA state moves to the next tile
    if (has_next) {
      tile_mn(npid, ntm, ntn);
      dma_init(da, db, ntm, ntn);
    }
    if constexpr (ZOP) {
      zr0 = tm * BM + wr * RW + (lane & 15);
      zc0 = tn * BN + wc * CW + 4 * (lane >> 4);
      zld = epi_scales(E) ? ldz : ldc;
      zp = (epi_scales(E) ? Z : C) + (int64_t)(zr0 < M ? zr0 : 0) * zld + zc0;
    }
    kstep(nk - 2, std::false_type{}, std::false_type{}, false, has_next, true, std::false_type{});
    kstep(nk - 1, std::false_type{}, std::false_type{}, false, has_next, false, std::true_type{});

    // ---- epilogue from registers: acc[i][j][r] = C[m0 + wr*RW + i*16 + (lane&15)][n0 + wc*CW + j*16 + 4*(lane>>4) + r]
    if constexpr (AGPR_ACC) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    const int m0 = tm * BM, n0 = tn * BN;
    const int lrow = lane & 15, g = lane >> 4;
    const int rb = m0 + wr * RW + lrow;
    const int cbase = n0 + wc * CW;
    // after the swap a lane holds 8 consecutive columns of block jp + ((lane >> 4) & 1)
    const int sw_col = ((lane >> 4) & 1) * 16 + 8 * (lane >> 5);
    // this lane's 4 bias values per block, packed (unpacked where used); weight gradients
    // (xᵀ·dy) and the scaling dgrad epilogues never carry a bias: no registers for it there
    constexpr bool HB = !DG && (AK || BK);
    uint2 bvp[HB ? TJ : 1];
#pragma unroll
    for (int j = 0; j < (HB ? TJ : 1); ++j) {
      const int n = cbase + j * 16 + 4 * g;
      bvp[j] = make_uint2(0u, 0u);
      if (HB && bias && n < N) bvp[j] = *reinterpret_cast<const uint2*>(bias + n);
    }
    // The scaling (dgrad) epilogues walk the tile in NH column passes so that only TJ / NH blocks'
    // column sums are live at a time (all TJ of them pushed the kernel past 256 VGPRs: per-tile
    // scratch spills of loop-invariant state).
#pragma unroll
    for (int hp = 0; hp < NH; ++hp) {
      float cs[JH][4];
#pragma unroll
      for (int j = 0; j < JH; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        __builtin_amdgcn_sched_barrier(0);  // one 16-row block at a time (ring loads stay in place; no accumulator hoisting)
        const int m = rb + i * 16;
        const bool mok = m < M;
        const float mk = (mok || (nts & 4)) ? 1.f : 0.f;
        const int64_t mr = mok ? m : 0;
        if constexpr (ZOP) {
          // ring: pass-row q + ZR - 1's loads go out before pass-row q is consumed
#pragma unroll
          for (int j = 0; j < JH; ++j) zload((hp * TI + i + ZR - 1) * JH + j);
        }
#pragma unroll
        for (int jq = 0; jq < JH; jq += 2) {
          const int jp = hp * JH + jq;
          uint2 gz[2];
          if constexpr (ZOP) {
            gz[0] = gza[(hp * TI + i) % ZR][jq];
            gz[1] = gza[(hp * TI + i) % ZR][jq + 1];
          }
          uint32_t pc[2][2], pz[2][2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int j = jp + u;
            // (the scaling epilogues are dgrads: no bias term)
            float v[4];
            if constexpr (DG) {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r];
            } else if constexpr (HB) {
              v[0] = acc[i][j][0] + to_f<T>(bvp[j].x & 0xffff);
              v[1] = acc[i][j][1] + to_f<T>(bvp[j].x >> 16);
              v[2] = acc[i][j][2] + to_f<T>(bvp[j].y & 0xffff);
              v[3] = acc[i][j][3] + to_f<T>(bvp[j].y >> 16);
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r];
            }
            if constexpr (DG) {
              const float z[4] = {to_f<T>(gz[u].x & 0xffff), to_f<T>(gz[u].x >> 16), to_f<T>(gz[u].y & 0xffff),
                                  to_f<T>(gz[u].y >> 16)};
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] *= zfac<E>(z[r]);
              // bias-gradient column sums of the fp32 products (rows past M contribute zeros:
              // a 0 / 1 factor per row block instead of a select per element; those rows hold
              // finite copies of row M-1, the operand DMA clamps them)
              if (nts & 4) {  // (A/B: the per-element select form)
                if (mok) {
#pragma unroll
                  for (int r = 0; r < 4; ++r) cs[jq + u][r] += v[r];
                }
              } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) cs[jq + u][r] = fmaf(v[r], mk, cs[jq + u][r]);
              }
            } else if constexpr (epi_gd(E)) {
              float d[4];
              // (nts bit 2: the scalar form, A/B)
              if (!(nts & 4)) {
                pf32x2 d01, d23;
                const pf32x2 y01 = E == kGeluTanhD ? gelu_tanh_d2(pf32x2{v[0], v[1]}, d01)
                                                   : gelu_erf_d2(pf32x2{v[0], v[1]}, d01);
                const pf32x2 y23 = E == kGeluTanhD ? gelu_tanh_d2(pf32x2{v[2], v[3]}, d23)
                                                   : gelu_erf_d2(pf32x2{v[2], v[3]}, d23);
                v[0] = y01.x, v[1] = y01.y, v[2] = y23.x, v[3] = y23.y;
                d[0] = d01.x, d[1] = d01.y, d[2] = d23.x, d[3] = d23.y;
              } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = act_d<E>(v[r], d[r]);
              }
              pz[u][0] = pack2<T>(d[0], d[1]);
              pz[u][1] = pack2<T>(d[2], d[3]);
            } else if constexpr (E != kNone) {
              pz[u][0] = pack2<T>(v[0], v[1]);
              pz[u][1] = pack2<T>(v[2], v[3]);
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = act<E>(v[r]);
            }
            if constexpr (BETA && !DG) {
              v[0] += to_f<T>(gz[u].x & 0xffff);
              v[1] += to_f<T>(gz[u].x >> 16);
              v[2] += to_f<T>(gz[u].y & 0xffff);
              v[3] += to_f<T>(gz[u].y >> 16);
            }
            pc[u][0] = pack2<T>(v[0], v[1]);
            pc[u][1] = pack2<T>(v[2], v[3]);
          }
          // rows 1 and 3 (lanes 16-31, 48-63) take block jp+1's first 4 columns from rows 0 / 2,
          // which take block jp's last 4 columns: every lane then holds 8 consecutive columns
          const int nc = cbase + jp * 16 + sw_col;
          {
            auto r0 = __builtin_amdgcn_permlane16_swap(pc[0][0], pc[1][0], false, false);
            auto r1 = __builtin_amdgcn_permlane16_swap(pc[0][1], pc[1][1], false, false);
            if (mok && nc < N) {
              const u32x4 w = {r0[0], r1[0], r0[1], r1[1]};
              if (nts & 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(C + mr * ldc + nc), "v"(w) : "memory");
              else *reinterpret_cast<u32x4*>(C + mr * ldc + nc) = w;
            }
          }
          if constexpr (!DG && E != kNone) {
            if (Z) {
              auto r0 = __builtin_amdgcn_permlane16_swap(pz[0][0], pz[1][0], false, false);
              auto r1 = __builtin_amdgcn_permlane16_swap(pz[0][1], pz[1][1], false, false);
              if (mok && nc < N) {
                const u32x4 w = {r0[0], r1[0], r0[1], r1[1]};
                if (nts & 2) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(Z + mr * ldz + nc), "v"(w) : "memory");
                else *reinterpret_cast<u32x4*>(Z + mr * ldz + nc) = w;
              }
            }
          }
        }
      }
      if constexpr (DG) {
        if (colsum) {
          // lanes with equal lane >> 4 own the same 4 columns of each block: reduce over lane & 15
          // (one DPP row: row_shr 1/2/4/8 inclusive scan, lane 15 of the row ends with the total;
          // v_add_f32_dpp, no ds_bpermute), lane 15 parks the pass's sums in its wave row's LDS row
#pragma unroll
          for (int j = 0; j < JH; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) cs[j][r] = row16_sum(cs[j][r]);
          if (lrow == 15) {
#pragma unroll
            for (int j = 0; j < JH; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) xlds[wr * BN + wc * CW + (hp * JH + j) * 16 + 4 * g + r] = cs[j][r];
          }
        }
      }
    }
    if constexpr (DG) {
      if (colsum) {
        // the two wave rows' sums -> this tile's partial row (one column per thread, coalesced)
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();
        for (int t = tid; t < BN; t += NT)
          if (n0 + t < N) colsum[(int64_t)tm * N + n0 + t] = xlds[t] + xlds[BN + t];
      }
    }
    if (!has_next) break;
    // the next tile's step 0 landed in slot 0 before the last K-step's second barrier: its first
    // fragments are read only now, so they do not occupy registers through the epilogue
#pragma unroll
    for (int j = 0; j < TJ; ++j) fb0[j] = frag<T, BK>(lds + IMGA, wc * CW + j * 16, 0, lane);
#pragma unroll
    for (int i = 0; i < TI; ++i) fa0[i] = frag<T, AK, (AK ? 256 : BM)>(lds, wr * RW + i * 16, 0, lane);
    pid = npid;
    tm = ntm;
    tn = ntn;
  }
}

}  // namespace
}  // namespace pra
