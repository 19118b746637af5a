// capgen — the bf16 MFMA GEMM tile (LDS-DMA ring, k-loop, epilogue, in-launch split-K) as device
// code shared by the plain and the grouped GEMM launches (gemm_bf16.hip).  Design notes:
// gemm_bf16.hip header.
#pragma once
#include "gemm.h"

namespace capgen {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;
typedef __attribute__((address_space(3))) void lds_void;

namespace {

constexpr int BK = 64;


// swizzles (16-B chunk index permutations, involutions)
// [row][64 k]: key ((row>>1) ^ (row>>4)) & 7 is a bijection on any 16 aligned rows (conflict-free
// ds_read_b64 fragments) AND differs between rows r and r+16, so hipcc cannot fuse two
// fragments' reads into a ds_read2st64_b64 (mod-32 banking: 2-way conflicts)
__device__ __forceinline__ int swz_k(int row, int chunk) { return chunk ^ (((row >> 1) ^ (row >> 4)) & 7); }
template <int ROWS>
__device__ __forceinline__ int swz_t(int k, int chunk) {                                   // [k][ROWS]
  if constexpr (ROWS == 128) return chunk ^ ((k & 7) << 1);
  else if constexpr (ROWS == 64) return chunk ^ (((k >> 1) & 3) << 1);
  else return chunk ^ (((k >> 2) & 1) << 1);  // 32 rows = 4 chunks per K row
}

template <bool TRANS, int ROWS, int NW>
struct Op {
  static constexpr int BYTES = ROWS * BK * 2;   // one stage of this operand
  static constexpr int NI = BYTES / 1024;       // 1-KB DMA instructions per stage
  static constexpr int PER_WAVE = NI / NW;
  static_assert(PER_WAVE >= 1 && NI % NW == 0, "tile too small for the wave count");
  static constexpr uint32_t OOB = 0x80000000u;  // past any buffer: the DMA lands zeros

  // The operand is read through a buffer resource (bounds-checked: an offset past num_records
  // returns zeros), so the k-loop issues each 1-KB piece with NO per-piece address arithmetic:
  // every lane's byte offset is fixed for the tile (voff, set up once) and the k-tile advance is
  // one scalar soffset (kstep per tile).  Nothing is left to num_records: a chunk outside the
  // tile's extent (non-TRANS: rows >= R; TRANS: columns >= R) gets the OOB offset once, and the
  // K tail (non-TRANS: k columns >= K; TRANS: k rows >= K) is masked per lane on the last
  // k-tile.  (The first version left the TRANS k rows >= K of a tile with soff > 0 to the range
  // check: the bf16 step's encoder weight gradients -- K = 72 tokens, two k-tiles -- then
  // differed between identical runs in 9 of 16 probes, 0 of 16 with the mask,
  // tools/step_det_probe.py; a standalone GEMM over NaN-poisoned neighbours did not show it.)
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t voff[PER_WAVE];
  int kch[PER_WAVE];  // k offset of the lane's chunk (non-TRANS: column, TRANS: row) in the tile
  uint32_t kstep;

  __device__ __forceinline__ void setup(const bf16* src, int64_t ld, int r0, int R, int K, int kt_first, int wave,
                                        int lane) {
    const int64_t rows = TRANS ? K : R;
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(src), 0, (int)(rows * ld * 2), 0x00020000);
    kstep = TRANS ? (uint32_t)(BK * ld * 2) : (uint32_t)(BK * 2);
#pragma unroll
    for (int j = 0; j < PER_WAVE; ++j) {
      const int i = wave + NW * j;
      const int b = i * 1024 + lane * 16;
      if constexpr (!TRANS) {
        const int row = b >> 7, ch = swz_k(row, (b >> 4) & 7);
        kch[j] = ch * 8;
        voff[j] = r0 + row < R ? (uint32_t)(((int64_t)(r0 + row) * ld + (int64_t)kt_first * BK + ch * 8) * 2) : OOB;
      } else {
        const int k = b / (ROWS * 2), ch = swz_t<ROWS>(k, (b % (ROWS * 2)) >> 4);
        kch[j] = k;
        voff[j] = r0 + ch * 8 < R ? (uint32_t)((((int64_t)kt_first * BK + k) * ld + r0 + ch * 8) * 2) : OOB;
      }
    }
  }

  // this wave's share of the LDS-DMA for k-tile t (relative to kt_first) into the stage image
  // img; tail: the tile ends past K (kb = its first k)
  __device__ __forceinline__ void issue(int t, char* img, bool tail, int kb, int K, int wave) const {
    const uint32_t soff = (uint32_t)t * kstep;
    if (tail) {  // uniform: the last k-tile of a K that is not a multiple of 64
#pragma unroll
      for (int j = 0; j < PER_WAVE; ++j) dma(kb + kch[j] < K ? voff[j] : OOB, soff, img + (wave + NW * j) * 1024);
    } else {
#pragma unroll
      for (int j = 0; j < PER_WAVE; ++j) dma(voff[j], soff, img + (wave + NW * j) * 1024);
    }
  }

  // one 1-KB LDS-DMA piece (buffer_load_dwordx4 ... lds: lane l's 16 B land at M0 + 16 l), issued
  // by inline asm.  With the global_load_lds builtin hipcc treated the in-flight DMA as a pending
  // write to the staging array and emitted `s_waitcnt vmcnt(0)` before the next ds_read of ANY
  // stage, draining every prefetch one step early (guide cdna_hip_programming.md §5 item 4(a));
  // the k-loop retires the DMA itself with counted vmcnt waits + a raw barrier (wait_younger).
  // `s_nop 4` opens the statement: hipcc pads no hazard into or out of an asm string, and the
  // descriptor / soffset SGPRs may come straight from a VALU write (v_readlane when hipcc restores
  // spilled SGPRs, v_readfirstlane) -- VALU-writes-SGPR -> VMEM-reads-it needs 5 wait states, and
  // the M0 write just before the statement 1.  Without them the DMA read a stale descriptor: the
  // round-4 persistent FFN's wrong W2 tiles (a kernel whose SGPR pressure made hipcc restore the W2
  // operand's descriptor by v_readlane right before the DMA; tools/persist_ffn.py).
  __device__ __forceinline__ void dma(uint32_t v, uint32_t soff, char* lds) const {
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(v), "s"(rsrc), "s"(soff),
                 "{m0}"((unsigned)(uintptr_t)lds)
                 : "memory");
  }

  // 16-row fragment starting at rb for k-step ks (permuted K order, see header)
  static __device__ __forceinline__ bf16x8 frag(const char* img, int rb, int ks, int lane) {
    const int g = lane >> 4;
    s4 lo, hi;
    if constexpr (!TRANS) {
      const int row = rb + (lane & 15);
      const int c1 = ks * 4 + (g >> 1), sub = (g & 1) * 8;
      lo = *reinterpret_cast<const s4*>(img + row * 128 + swz_k(row, c1) * 16 + sub);
      hi = *reinterpret_cast<const s4*>(img + row * 128 + swz_k(row, c1 + 2) * 16 + sub);
    } else {
      const int i = lane & 15, q = i >> 2, p = i & 3;
      const int k = ks * 32 + 4 * g + q;
      const int ch = (rb >> 3) + (p >> 1), sub = (p & 1) * 8;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s4*)(img + k * (ROWS * 2) + swz_t<ROWS>(k, ch) * 16 + sub));
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s4*)(img + (k + 16) * (ROWS * 2) + swz_t<ROWS>(k + 16, ch) * 16 + sub));
    }
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most min(younger, MAXY) K tiles' DMA (LPT instructions each) are in flight
template <int LPT, int MAXY>
__device__ __forceinline__ void wait_younger(int younger) {
  if constexpr (MAXY == 0) {
    wait_vmcnt<0>();
  } else {
    if (younger >= MAXY) wait_vmcnt<MAXY * LPT>();
    else wait_younger<LPT, MAXY - 1>(younger);
  }
}

template <typename TO>
__device__ __forceinline__ void load4(const TO* p, float (&v)[4]) {
  if constexpr (sizeof(TO) == 4) {
    float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w;
  } else {
    typedef __attribute__((ext_vector_type(4))) __bf16 b4;
    b4 x = *reinterpret_cast<const b4*>(p);
    v[0] = (float)x[0], v[1] = (float)x[1], v[2] = (float)x[2], v[3] = (float)x[3];
  }
}
template <typename TO>
__device__ __forceinline__ void store4(TO* p, const float (&v)[4]) {
  if constexpr (sizeof(TO) == 4) {
    *reinterpret_cast<float4*>(p) = float4{v[0], v[1], v[2], v[3]};
  } else {
    typedef __attribute__((ext_vector_type(4))) __bf16 b4;
    *reinterpret_cast<b4*>(p) = b4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  }
}

}  // namespace

// Tile geometry of one variant (shared by the plain and the grouped launch).  KG k-groups: the
// workgroup holds KG groups of WM x WN waves; group g runs the k-loop over the g-th contiguous
// chunk of the tile's k-tiles with its own LDS ring (the per-workgroup k-chain is latency-bound --
// tools/gemm_phase_timing.py: ~1000 cycles per 64-deep step of a 64x64 tile, time independent of M
// -- so KG chains of nk/KG steps run side by side on the same CU), then the groups sum their
// partial tiles through LDS in group order (bit-identical to grid split-K with KG slices) and each
// group stores 1/KG of the tile's fragments.
template <bool TA, bool TB, int BM, int BN, int WM, int WN, int STAGES, int KG = 1>
struct TileCfg {
  static constexpr int NW = WM * WN;  // waves per k-group
  static constexpr int NWT = NW * KG;  // waves per workgroup
  typedef Op<TA, BM, NW> OA;
  typedef Op<TB, BN, NW> OB;
  static constexpr int SB = OA::BYTES + OB::BYTES;  // LDS bytes per stage
  static constexpr int XCH = KG > 1 ? (BM / WM / 16) * (BN / WN / 16) * KG * NW * 64 * 16 : 0;  // k-group exchange
  static constexpr int SMEM = KG * STAGES * SB > XCH ? KG * STAGES * SB : XCH;
};

template <typename TO, int FM, int FN, int TM, int TN>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& g, const f32x4 (&acc)[FM][FN], int m0, int n0, int wm,
                                              int wn, int lane, float alpha, int kgrp = 0, int kgs = 1);

// Diagnostic ablation build (make ablate -> libcapgen_ablate.so, tools/gemm_ablate.py): protocol bit
// 1024 skips the MFMAs, bit 2048 skips the operand DMA and its waits -- what a shape costs without
// its arithmetic, without its operand ingest, or with neither (the launch + epilogue intercept).
// Bit 4096 (same build): wave 0 of block 0 records s_memtime / s_memrealtime at the kernel start, after
// the prologue DMA issue, at four points of each of the first 8 k-steps (after the DMA wait, after
// the barrier, after the next stage's DMA issue, after the MFMAs) and after the epilogue, into
// g.stamp[16 ..] (gemm_set_timing_buf): cycles per phase and the in-kernel clock.
#ifdef CAPGEN_GEMM_ABLATE
#define ABL_NO_MFMA (proto & 1024)
#define ABL_NO_DMA (proto & 2048)
#define ABL_DMA_FIRST (proto & 8192)  // 4-wave tiles take the DMA-issue-first k-step order too
#define ABL_T(slot)                                                                                   \
  do {                                                                                                \
    if ((proto & 4096) && g.stamp && blockIdx.x == 0 && threadIdx.x == 0) {                           \
      g.stamp[16 + 2 * (slot)] = __builtin_amdgcn_s_memtime();                                        \
      g.stamp[17 + 2 * (slot)] = __builtin_amdgcn_s_memrealtime();                                    \
    }                                                                                                 \
  } while (0)
#else
#define ABL_NO_MFMA 0
#define ABL_NO_DMA 0
#define ABL_DMA_FIRST 0
#define ABL_T(slot) \
  do {              \
  } while (0)
#endif

// diagnostic counters of the split-K hand-off (protocol bit 64): [0] tickets found >= splitk at
// arrival (a ticket not re-armed before this launch), [1] tiles combined
static __device__ int g_sk_diag[4];  // (per translation unit)

// One BMxBN output tile (split-K slice `split` of `splitk`) of C = op(A).op(B): the LDS-DMA
// ring, the MFMA main loop and the epilogue (in-launch split-K combine included).
template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int STAGES, int KG = 1>
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, int mt, int nt, int tile, int split, int splitk,
                                          const void* zero, float* ws, int* tile_cnt, char* smem, int proto = 0) {
  typedef TileCfg<TA, TB, BM, BN, WM, WN, STAGES, KG> Cfg;
  constexpr int NW = Cfg::NW;
  typedef typename Cfg::OA OA;
  typedef typename Cfg::OB OB;
  constexpr int SB = Cfg::SB;                       // bytes per stage
  constexpr int LPT = OA::PER_WAVE + OB::PER_WAVE;  // DMA instructions per wave per K tile
  constexpr int TM = BM / WM, TN = BN / WN;         // per-wave tile
  constexpr int FM = TM / 16, FN = TN / 16;
  static_assert(STAGES >= 2, "need >= 2 stages");
  const int m0 = mt * BM, n0 = nt * BN;

  ABL_T(0);
  const bf16* __restrict__ A = reinterpret_cast<const bf16*>(g.A);
  const bf16* __restrict__ B = reinterpret_cast<const bf16*>(g.B);
  const int lane = threadIdx.x & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kgrp = KG > 1 ? wave_all / NW : 0;  // k-group of this wave
  const int wave = KG > 1 ? wave_all % NW : wave_all;
  const int wm = wave / WN, wn = wave % WN;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk_all = (g.K + BK - 1) / BK;
  const int per = (nk_all + splitk - 1) / splitk;
  const int nks = max(0, min(nk_all - split * per, per));  // K tiles of this slice
  const int per_g = (nks + KG - 1) / KG;                    // ... of each k-group (the loop's trip count)
  const int kt0 = split * per + kgrp * per_g;               // this group's first k-tile
  const int nk = max(0, min(nks - kgrp * per_g, per_g));    // this group's k-tiles (<= per_g)
  if (KG > 1) smem += kgrp * (STAGES * SB);                 // the group's LDS ring
  OA oa;
  OB ob;
  oa.setup(A, g.lda, m0, g.M, g.K, kt0, wave, lane);
  ob.setup(B, g.ldb, n0, g.N, g.K, kt0, wave, lane);
  auto issue = [&](int t, char* st) {
    if (ABL_NO_DMA) return;
    const int kb = (kt0 + t) * BK;
    const bool tail = kb + BK > g.K;
    oa.issue(t, st, tail, kb, g.K, wave);
    ob.issue(t, st + OA::BYTES, tail, kb, g.K, wave);
  };
#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < nk) issue(p, smem + p * SB);
  ABL_T(1);

  // k-loop unrolled by STAGES: tile kb + s lives in stage s, so every LDS offset is a constant
  // (ds_read immediate offsets, a scalar M0 per DMA piece: no address VALU in the loop)
  static_assert((STAGES - 2) * LPT <= 63, "vmcnt range");
  // (every k-group runs per_g trips -- the barriers stay uniform -- and works on its own nk)
  for (int kb = 0; kb < per_g; kb += STAGES) {
#pragma unroll
    for (int s = 0; s < STAGES; ++s) {
      const int kt = kb + s;
      if (kt < per_g) {
        const bool work = KG == 1 || kt < nk;
        // tile kt landed for this wave (up to STAGES-2 younger tiles may still fly) ...
        if (!ABL_NO_DMA && work) wait_younger<LPT, STAGES - 2>(nk - 1 - kt);
        if (kt < 8) ABL_T(2 + 4 * kt);
        __builtin_amdgcn_s_barrier();  // ... for every wave; stage (s-1) % STAGES is free again
        if (kt < 8) ABL_T(3 + 4 * kt);
        const char* st = smem + s * SB;
        if (NW * KG > 4 || ABL_DMA_FIRST) {
          // 8- and 16-wave tiles (and k-group tiles): DMA issue, then per 32-deep step its fragment
          // reads + MFMAs (hipcc reuses the fragment registers across the two steps).  Measured
          // against the read-everything-first order below (tools/gemm_splitk_sweep.py, r03): that
          // order is 1-4 % faster for one-wave-per-SIMD 4-wave tiles and 2-30 % slower here.
          if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, smem + ((s + STAGES - 1) % STAGES) * SB);
          if (kt < 8) ABL_T(4 + 4 * kt);
#pragma unroll
          for (int ks = 0; ks < BK / 32; ++ks) {
            if (!work) break;
            bf16x8 af[FM], bfr[FN];
#pragma unroll
            for (int i = 0; i < FM; ++i) af[i] = OA::frag(st, wm * TM + i * 16, ks, lane);
#pragma unroll
            for (int j = 0; j < FN; ++j) bfr[j] = OB::frag(st + OA::BYTES, wn * TN + j * 16, ks, lane);
            if (ABL_NO_MFMA) {  // (ablation: keep the fragment reads live)
#pragma unroll
              for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j) acc[i][j][0] += (float)af[i][0] + (float)bfr[j][0];
              continue;
            }
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
              for (int j = 0; j < FN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
          }
        } else {
          // Every fragment read of the k-tile (both 32-deep steps, distinct registers) is issued
          // first, then the next stage's DMA, then the MFMAs in read order: hipcc's counted
          // lgkmcnt waits let each MFMA start as soon as its own two fragments land, and the DMA
          // issue (~270 cycles, tools/gemm_phase_timing.py) overlaps the LDS read latency.  At one
          // wave per SIMD the LDS only reaches its rate with reads kept in flight (MI355X_MICROARCH.md
          // §LDS: a wave that drains after each short group gets a fifth of it).
          constexpr int KS = BK / 32;
          bf16x8 af[KS][FM], bfr[KS][FN];
          if (work) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
              for (int i = 0; i < FM; ++i) af[ks][i] = OA::frag(st, wm * TM + i * 16, ks, lane);
#pragma unroll
              for (int j = 0; j < FN; ++j) bfr[ks][j] = OB::frag(st + OA::BYTES, wn * TN + j * 16, ks, lane);
            }
          }
          // (the DMA targets stage (s-1) % STAGES, freed by the barrier; the reads above are of stage s)
          if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, smem + ((s + STAGES - 1) % STAGES) * SB);
          if (kt < 8) ABL_T(4 + 4 * kt);
          if (work) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              if (ABL_NO_MFMA) {  // (ablation: keep the fragment reads live)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                  for (int j = 0; j < FN; ++j) acc[i][j][0] += (float)af[ks][i][0] + (float)bfr[ks][j][0];
                continue;
              }
#pragma unroll
              for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                  acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
            }
          }
        }
        if (kt < 8) ABL_T(5 + 4 * kt);
      }
    }
  }
  ABL_T(34);

  // ---- epilogue: lane holds C[m = mb + (lane&15)][n = nb + 4*(lane>>4) + 0..3] ----
  const float alpha = g.alpha_ptr ? g.alpha * *g.alpha_ptr : g.alpha;
  if constexpr (KG > 1) {
    // k-group exchange: fragment f = i * FN + j belongs to group f % KG; every group parks the
    // fragments it does not own in LDS (the rings are idle: every DMA was waited for, every
    // fragment read consumed), then each owner sums the KG partials in group order
    if (KG > 1) smem -= kgrp * (STAGES * SB);
    f32x4* ex = reinterpret_cast<f32x4*>(smem);
    constexpr int NF = FM * FN;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        if ((i * FN + j) % KG != kgrp) ex[(((i * FN + j) * KG + kgrp) * NW + wave) * 64 + lane] = acc[i][j];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if ((i * FN + j) % KG != kgrp) continue;
        f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h = 0; h < KG; ++h) sum += h == kgrp ? acc[i][j] : ex[(((i * FN + j) * KG + h) * NW + wave) * 64 + lane];
        acc[i][j] = sum;
      }
    tile_epilogue<TO, FM, FN, TM, TN>(g, acc, m0, n0, wm, wn, lane, alpha, kgrp, KG);
    ABL_T(35);
    return;
  }
  if (splitk > 1) {
    // Split-K combine inside the launch (the guide's counter hand-off, cdna_hip_programming.md
    // §5 'Projection GEMM' item 2 / §6 Guideline 16): every slice stores its raw partial tile
    // to the f32 workspace with 16-B write-through (sc1) buffer stores (no release fence
    // needed), every wave drains them (vmcnt(0)), the workgroup barrier, then ONE lane takes a
    // ticket (agent atomic).  The block that draws the last ticket re-arms the ticket with an
    // atomic exchange (performed where the adds are: a plain or sc1 store of 0 mixed with the
    // atomic adds made later launches miscount, tools/step_det_probe.py) and runs ONE
    // agent-scope acquire (drops this CU's stale L1 lines: several workgroups share a CU here)
    // before any wave reads the other slices; it sums all slices in slice order (deterministic
    // whichever block is last) and runs the normal epilogue.  Correct for any placement of a
    // tile's slices over CUs / XCDs.
    // `proto` (diagnostic, capgen_debug_splitk_protocol): bit 0 adds a writer release, bit 1
    // drops the reader acquire, bit 2 reads the slabs with sc1 loads, bit 4 re-arms the ticket
    // with a relaxed atomic store (the round-1 form was bits 1|2|4); bit 3 is the launcher's
    // per-launch ticket memset.
    constexpr int NT = 64 * NW, NF = FM * FN;
    const int tid = threadIdx.x;
    const int64_t tile_bytes = (int64_t)splitk * NF * NT * 16;
    char* tbase = reinterpret_cast<char*>(ws) + (int64_t)tile * tile_bytes;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(tbase, 0, (int)tile_bytes, 0x00020000);
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        if (proto & 512)  // diagnostic: system-scope (sc0 sc1) slab stores
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rsrc,
                                                 ((split * NF + i * FN + j) * NT + tid) * 16, 0, 17);
        else
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rsrc,
                                                 ((split * NF + i * FN + j) * NT + tid) * 16, 0, 16 /* sc1 */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    typedef __attribute__((address_space(3))) volatile int lds_int;
    lds_int* flag = (lds_int*)smem;  // staging LDS is free now
    if (tid == 0) {
      if (proto & 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fence's own wait can be dropped (G16 pitfall 12)
      }
      const int old = __hip_atomic_fetch_add(tile_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == splitk - 1;
      if (proto & 64) {
        if (old < 0 || old >= splitk) atomicAdd(&g_sk_diag[0], 1);
        if (last) atomicAdd(&g_sk_diag[1], 1);
      }
      if (last) {
        if (proto & 16) __hip_atomic_store(tile_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else (void)__hip_atomic_exchange(tile_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (proto & 128) {  // diagnostic: system-scope acquire
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (!(proto & 2)) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // holds the barrier below until the invalidate is done
        }
      }
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the ticket
    const int lpol = (proto & 256) ? 17 : (proto & 4) ? 16 /* sc1 */ : 0;
    // slice by slice in slice order (deterministic, and the k-group exchange's order: 0 + p0 + p1 + ...);
    // every fragment's load of one slice is issued before any is used (one round trip per slice, not
    // per slice and fragment)
    f32x4 sum[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) sum[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sl = 0; sl < splitk; ++sl) {
      if (sl == split) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) sum[i][j] += acc[i][j];
        continue;
      }
      u32x4 o[FM][FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int off = ((sl * NF + i * FN + j) * NT + tid) * 16;
          o[i][j] = lpol == 17 ? __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 17)
                    : lpol     ? __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 16)
                               : __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
        }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) sum[i][j] += __builtin_bit_cast(f32x4, o[i][j]);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = sum[i][j];
  }
  tile_epilogue<TO, FM, FN, TM, TN>(g, acc, m0, n0, wm, wn, lane, alpha);
  ABL_T(35);
}

// Store one tile's accumulators: alpha, bias, ReLU' mask (aux), ReLU, accumulate (beta),
// conversion, column sums.  Lane holds C[m = mb + (lane&15)][n = nb + 4*(lane>>4) + 0..3].
template <typename TO, int FM, int FN, int TM, int TN>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& g, const f32x4 (&acc)[FM][FN], int m0, int n0, int wm,
                                              int wn, int lane, float alpha, int kgrp, int kgs) {
  TO* __restrict__ C = reinterpret_cast<TO*>(g.C);
  TO* __restrict__ C2 = reinterpret_cast<TO*>(g.C2);
  const bf16* __restrict__ aux = reinterpret_cast<const bf16*>(g.aux);
  const __amdgpu_buffer_rsrc_t crs = wt_rsrc(g.C);
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (sizeof(TO) == 2) {
    if (g.ce_stats) {  // fused cross-entropy epilogue (GemmArgs::ce_stats)
      // a 16x16 fragment = 16 rows x one 16-column slab; the 4 lanes of a row (lane groups fq)
      // hold its 4 column quads, so slab max / sum are two xor-shuffles.  Every lane runs the
      // shuffles (partners share the row, so out-of-range rows only predicate the stores).
      // every bias / target load first (clamped addresses, unconditional): one round trip
      float4 bq[FN];
      int tgq[FM];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = min(n0 + wn * TN + j * 16 + fq * 4, g.N - 4);
        bq[j] = g.bias ? *reinterpret_cast<const float4*>(g.bias + n) : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) tgq[i] = g.ce_tgt[min(m0 + wm * TM + i * 16 + fr, g.M - 1)];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + wm * TM + i * 16 + fr;
        const bool mok = m < g.M;
        const int tg = mok ? tgq[i] : -1;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if ((i * FN + j) % kgs != kgrp) continue;  // (k-groups: another group stores it)
          const int nb = n0 + wn * TN + j * 16, n = nb + fq * 4;
          const bool nok = n < g.N;
          float v[4], mx = -INFINITY;
          if (nok) {
            const float4 b4 = bq[j];
            v[0] = alpha * acc[i][j][0] + b4.x, v[1] = alpha * acc[i][j][1] + b4.y;
            v[2] = alpha * acc[i][j][2] + b4.z, v[3] = alpha * acc[i][j][3] + b4.w;
            mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
          }
          mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
          mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
          float e[4], sum = 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            e[r] = nok ? __expf(v[r] - mx) : 0.f;
            sum += e[r];
          }
          sum += __shfl_xor(sum, 16, 64);
          sum += __shfl_xor(sum, 32, 64);
          if (mok && nok) {
            store4<TO>(C + (int64_t)m * g.ldc + n, e);
            if (tg >= n && tg < n + 4) g.ce_tlogit[m] = v[tg - n];
          }
          if (mok && fq == 0 && nb < g.N) g.ce_stats[(int64_t)m * g.ce_ld + nb / 16] = float2{mx, sum};
        }
      }
      return;
    }
  }
  if constexpr (sizeof(TO) == 4) {
    if (g.dec_stats) {  // decode classifier epilogue (GemmArgs::dec_stats): f32 logits + slab stats
      // same fragment geometry as the cross-entropy epilogue above: the 4 lane groups of a row hold
      // its 16-column slab, so the slab max / exp-sum are two xor-shuffles
      float4 bq[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = min(n0 + wn * TN + j * 16 + fq * 4, g.N - 4);
        bq[j] = g.bias ? *reinterpret_cast<const float4*>(g.bias + n) : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + wm * TM + i * 16 + fr;
        const bool mok = m < g.M;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if ((i * FN + j) % kgs != kgrp) continue;
          const int nb = n0 + wn * TN + j * 16, n = nb + fq * 4;
          const bool nok = n < g.N;
          float v[4], mx = -INFINITY;
          if (nok) {
            const float4 b4 = bq[j];
            v[0] = alpha * acc[i][j][0] + b4.x, v[1] = alpha * acc[i][j][1] + b4.y;
            v[2] = alpha * acc[i][j][2] + b4.z, v[3] = alpha * acc[i][j][3] + b4.w;
            mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
          }
          mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
          mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
          float sum = 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) sum += nok ? __expf(v[r] - mx) : 0.f;
          sum += __shfl_xor(sum, 16, 64);
          sum += __shfl_xor(sum, 32, 64);
          if (mok && nok) store4<TO>(C + (int64_t)m * g.ldc + n, v);
          if (mok && fq == 0 && nb < g.N) g.dec_stats[(int64_t)m * g.dec_ld + nb / 16] = float2{mx, sum};
        }
      }
      return;
    }
  }
  // Generic epilogue.  Every side-operand load of the tile (bias, ReLU' mask, the accumulated C) is
  // issued before the first store: the loads of one fragment used to wait for the previous fragment's
  // store (hipcc cannot move a load across a store in another basic block), one memory round trip per
  // fragment and operand -- the ReLU'-masked FFN input-gradient GEMMs ran at 2.5x their forward twins
  // in the step.  (The f32 cin operand of the removed split-encoder-gradient experiment is gone.)
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  float bn[FN][4];
  u32x2 auxr[FM][FN];          // 4 bf16 of the ReLU' mask
  float cold[FM][FN][4];       // beta: the C values accumulated into
  bool ok[FM][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * TN + j * 16 + fq * 4;
    const bool nok = n < g.N;
    float4 b4 = float4{0.f, 0.f, 0.f, 0.f};
    if (g.bias && nok) b4 = *reinterpret_cast<const float4*>(g.bias + n);
    bn[j][0] = b4.x, bn[j][1] = b4.y, bn[j][2] = b4.z, bn[j][3] = b4.w;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * TM + i * 16 + fr;
      ok[i][j] = nok && m < g.M && (i * FN + j) % kgs == kgrp;
    }
  }
  if (aux) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int m = min(m0 + wm * TM + i * 16 + fr, g.M - 1), n = min(n0 + wn * TN + j * 16 + fq * 4, g.N - 4);
        auxr[i][j] = *reinterpret_cast<const u32x2*>(aux + (int64_t)m * g.ldaux + n);
      }
  }
  if (g.beta) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        // (clamped in-range address, loaded unconditionally: a load inside a per-fragment branch is
        // waited for at the branch's join)
        const int m = min(m0 + wm * TM + i * 16 + fr, g.M - 1), n = min(n0 + wn * TN + j * 16 + fq * 4, g.N - 4);
        const bool hi = C2 && n >= g.nsplit;
        const TO* cp = hi ? C2 + (int64_t)m * g.ldc2 + (n - g.nsplit) : C + (int64_t)m * g.ldc + n;
        load4<TO>(cp, cold[i][j]);
      }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * TN + j * 16 + fq * 4;
    float cs[4] = {0.f, 0.f, 0.f, 0.f};
    if (n >= g.N) continue;
    const bool hi = C2 && n >= g.nsplit;  // split output: this 4-column group goes to C2
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * TM + i * 16 + fr;
      if (!ok[i][j]) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = alpha * acc[i][j][r] + bn[j][r];
      if (aux) {
        const float a4[4] = {__uint_as_float(auxr[i][j][0] << 16), __uint_as_float(auxr[i][j][0] & 0xffff0000u),
                             __uint_as_float(auxr[i][j][1] << 16), __uint_as_float(auxr[i][j][1] & 0xffff0000u)};
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = a4[r] > 0.f ? v[r] : 0.f;
      }
      if (g.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      TO* cp = hi ? C2 + (int64_t)m * g.ldc2 + (n - g.nsplit) : C + (int64_t)m * g.ldc + n;
      if (g.beta) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += cold[i][j][r];
      }
      if (g.wt > 0 && !hi) {  // write-through (capgen_common.h wt_rsrc)
        const uint32_t off = (uint32_t)(((int64_t)m * g.ldc + n) * (int64_t)sizeof(TO));
        if constexpr (sizeof(TO) == 4) {
          wt_store16(crs, off, wt_u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                        __float_as_uint(v[3])});
        } else {
          typedef __attribute__((ext_vector_type(4))) __bf16 b4;
          const b4 x = b4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          wt_store8(crs, off, __builtin_bit_cast(wt_u32x2, x));
        }
      } else {
        store4<TO>(cp, v);
      }
      if (g.colsum) {  // column sums of the stored values (as rounded to TO), from registers
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[r] += (float)(TO)v[r];
      }
    }
    if (g.colsum) {
      // reduce over the 16 lanes (rows) sharing these 4 columns, one atomic per column
#pragma unroll
      for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[r] += __shfl_xor(cs[r], o, 64);
      if (fr == 0) {
        float* cdst = g.colsum + (int64_t)(blockIdx.x % g.colsum_stripes) * g.colsum_stride + n;
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(cdst + r, cs[r]);
      }
    }
  }
}

// XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> give them adjacent slots
__device__ __forceinline__ int xcd_slot(int bid, int nblk) {
  const int xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

}  // namespace capgen
