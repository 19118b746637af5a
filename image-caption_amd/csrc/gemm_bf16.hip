// capgen — bf16 MFMA GEMM for gfx950, all three training layouts in one kernel template.
//
//   NT (forward  X.W^T)    : A [M][K], B [N][K]   both K-contiguous
//   NN (input grad dY.W)   : A [M][K], B [K][N]   B row-contiguous   (TB)
//   TN (weight grad dY^T.X): A [K][M], B [K][N]   both row-contiguous (TA, TB)
//
// Data movement.  Every operand tile is moved HBM/L2 -> LDS by global_load_lds_dwordx4
// (LDS-DMA, no staging registers) in its NATIVE layout, three stages deep: the DMA for
// K-tile kt+2 is in flight while tile kt is multiplied, retired by a counted
// `s_waitcnt vmcnt(loads per tile)` + raw s_barrier (never vmcnt(0) in the loop).
// LDS-DMA writes lane-linearly, so the bank-conflict swizzles are applied to the
// per-lane SOURCE address and undone on the fragment read (same involution).
// Out-of-range rows / K columns read a device zero page (no OOB access, exact K tails).
//
// Fragments.  K-contiguous images (128-B rows) are read with two ds_read_b64, XOR-
// swizzled in 16-B chunks by ((row>>1)&7).  Row-contiguous images are read with two
// ds_read_b64_tr_b16 (CDNA4 LDS transpose read), XOR-swizzled per K row.  Within each
// 32-deep v_mfma_f32_16x16x32_bf16 step, lane group g = lane>>4 carries k = 4g..4g+3
// (elements 0-3) and 16+4g..16+4g+3 (elements 4-7) for BOTH operands — the same K
// permutation on A and B leaves the dot product unchanged and makes every tr read of a
// half-wave cover 8 consecutive K rows (conflict free).  NT, NN and TN therefore run at
// the same LDS cost.
//
// Epilogue.  The MFMA is issued as B.A (operands swapped) so each lane ends with 4
// CONSECUTIVE output columns of one row: bias/relu-mask/accumulate/convert are applied
// on 4-wide vectors and stored as one 8-B (bf16) or 16-B (f32) write.
//
// Tiles BMxBNx64, 256 threads = 2x2 wave64s; blocks remapped so consecutive tiles (sharing
// an A row-panel) land on the same XCD L2.
#include <chrono>
#include <algorithm>
#include <dlfcn.h>
#include <string>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "gemm.h"
#include "hazard.h"

namespace capgen {

void gemm_hz_regions(const GemmArgs& g, DType in, DType out, bool ta, bool tb, std::vector<hz::Rgn>& v);  // gemm.hip

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;
typedef __attribute__((address_space(3))) void lds_void;

namespace {

constexpr int BK = 64;

void* g_zero_page[64] = {};

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
  __device__ __forceinline__ void dma(uint32_t v, uint32_t soff, char* lds) const {
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(v), "s"(rsrc), "s"(soff),
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
#define ABL_T(slot) \
  do {              \
  } while (0)
#endif

// diagnostic counters of the split-K hand-off (protocol bit 64): [0] tickets found >= splitk at
// arrival (a ticket not re-armed before this launch), [1] tiles combined
__device__ int g_sk_diag[4];

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
        if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, smem + ((s + STAGES - 1) % STAGES) * SB);
        if (kt < 8) ABL_T(4 + 4 * kt);
        const char* st = smem + s * SB;
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
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int sl = 0; sl < splitk; ++sl) {
          if (sl == split) {
            sum += acc[i][j];
          } else {
            const int off = ((sl * NF + i * FN + j) * NT + tid) * 16;
            const u32x4 o = lpol == 17 ? __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 17)
                            : lpol     ? __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 16)
                                       : __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
            sum += __builtin_bit_cast(f32x4, o);
          }
        }
        acc[i][j] = sum;
      }
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
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + wm * TM + i * 16 + fr;
        const bool mok = m < g.M;
        const int tg = mok ? g.ce_tgt[m] : -1;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if ((i * FN + j) % kgs != kgrp) continue;  // (k-groups: another group stores it)
          const int nb = n0 + wn * TN + j * 16, n = nb + fq * 4;
          const bool nok = n < g.N;
          float v[4], mx = -INFINITY;
          if (nok) {
            const float4 b4 = g.bias ? *reinterpret_cast<const float4*>(g.bias + n) : float4{0.f, 0.f, 0.f, 0.f};
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
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * TN + j * 16 + fq * 4;
    float cs[4] = {0.f, 0.f, 0.f, 0.f};
    if (n >= g.N) continue;
    const bool hi = C2 && n >= g.nsplit;  // split output: this 4-column group goes to C2
    float bn[4] = {0.f, 0.f, 0.f, 0.f};
    if (g.bias) {
      float4 b4 = *reinterpret_cast<const float4*>(g.bias + n);
      bn[0] = b4.x, bn[1] = b4.y, bn[2] = b4.z, bn[3] = b4.w;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + wm * TM + i * 16 + fr;
      if (m >= g.M || (i * FN + j) % kgs != kgrp) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = alpha * acc[i][j][r] + bn[r];
      if (g.cin) {
        float c4[4];
        load4<float>(g.cin + (int64_t)m * g.ldcin + n, c4);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += c4[r];
      }
      if (aux) {
        float a4[4];
        load4<bf16>(aux + (int64_t)m * g.ldaux + n, a4);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = a4[r] > 0.f ? v[r] : 0.f;
      }
      if (g.relu) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      TO* cp = hi ? C2 + (int64_t)m * g.ldc2 + (n - g.nsplit) : C + (int64_t)m * g.ldc + n;
      if (g.beta) {
        float o[4];
        load4<TO>(cp, o);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += o[r];
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

template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int STAGES, int KG = 1>
__global__ void __launch_bounds__(64 * WM * WN * KG) gemm_bf16_kernel(GemmArgs g, int tiles_n, int nblk,
                                                                     const void* zero, int splitk, float* ws,
                                                                     int* tile_cnt, int group_m, int proto) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<TA, TB, BM, BN, WM, WN, STAGES, KG>::SMEM];
  StampScope stamp_scope(g.stamp);
  // critical-path launch (GemmArgs::prio): beside the side streams' weight-gradient / Adam waves
  // on the same CUs, the SIMD arbiter issues this kernel's instructions first
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  const int slot = xcd_slot(blockIdx.x, nblk);
  const int tile = slot / splitk, split = slot % splitk;  // split-K slices of a tile are adjacent
  // tiles in column-major groups of group_m tile rows: an XCD's contiguous slot range covers a
  // compact 2D block of the output (fewer distinct A row panels + B column panels per L2)
  int mt = tile / tiles_n, nt = tile % tiles_n;
  if (group_m > 1) {
    const int tiles_m = (g.M + BM - 1) / BM, per = group_m * tiles_n, first = (tile / per) * group_m;
    const int gsz = min(tiles_m - first, group_m), r = tile % per;
    mt = first + r % gsz, nt = r / gsz;
  }
  gemm_tile<TO, TA, TB, BM, BN, WM, WN, STAGES, KG>(g, mt, nt, tile, split, splitk, zero, ws, tile_cnt, smem, proto);
}

// Grouped launch: up to kMaxGroup independent GEMMs of one layout (e.g. every weight gradient
// of a transformer block), each with its own M/N/pointers, tiles laid out problem after
// problem; one launch instead of one per weight, and a grid that fills the chip.
// G < nblk: a capped grid, each workgroup looping over the tiles b, b + G, ... (G % 8 == 0
// keeps every iteration on the workgroup's XCD).
template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int STAGES>
__global__ void __launch_bounds__(64 * WM * WN) gemm_bf16_grouped_kernel(GemmGroup gg, int nblk, int G,
                                                                        const void* zero) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<TA, TB, BM, BN, WM, WN, STAGES>::SMEM];
  StampScope stamp_scope(gg.p[0].stamp);
  for (int b = blockIdx.x; b < nblk; b += G) {
    if (b != (int)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
    const int slot = xcd_slot(b, nblk);
    int q = 0;
    while (q + 1 < gg.n && slot >= gg.start[q + 1]) ++q;
    const int tile = slot - gg.start[q];
    const int mt = tile / gg.tiles_n[q], nt = tile % gg.tiles_n[q];
    gemm_tile<TO, TA, TB, BM, BN, WM, WN, STAGES>(gg.p[q], mt, nt, tile, 0, 1, zero, nullptr, nullptr, smem);
  }
}

// split-K f32 workspaces, one per stream (GEMMs on different streams may run concurrently)
struct Workspace {
  float* p = nullptr;
  size_t bytes = 0;
  int* cnt = nullptr;  // per-tile arrival counters (zero between launches)
};
constexpr int kMaxTiles = 1 << 16;
std::map<hipStream_t, Workspace> g_ws;
// split-K hand-off protocol (diagnostic; 0 = production, see gemm_tile): bit 0 writer release,
// bit 1 no reader acquire, bit 2 sc1 slab loads, bit 3 per-launch ticket memset, bit 4 ticket
// re-armed by a relaxed atomic store (round 1: 2|4|16)
int g_splitk_proto = [] {
  const char* e = std::getenv("CAPGEN_SPLITK_PROTO");
  return e ? std::atoi(e) : 0;
}();
std::mutex g_ws_mu;
uint64_t* g_timing_buf = nullptr;  // ablation build, protocol bit 4096 (gemm_set_timing_buf)

// make sure the stream's split-K workspace holds `bytes` (never called inside a capture)
void ensure_ws(hipStream_t s, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Workspace& w = g_ws[s];
  if (!w.cnt) {
    CAPGEN_HIP(hipMalloc(&w.cnt, kMaxTiles * sizeof(int)));
    // on the stream itself: a null-stream hipMemset is not ordered before work on the
    // (non-blocking) engine streams, and a split-K launch reading stale tickets combines the
    // wrong slices (seen as a rare train_step vs forward/backward mismatch)
    CAPGEN_HIP(hipMemsetAsync(w.cnt, 0, kMaxTiles * sizeof(int), s));
  }
  if (w.bytes >= bytes) return;
  // a grown workspace retires the old one without freeing it: a graph captured earlier on
  // this stream (the replayed forward) still holds its address
  static std::vector<float*> retired;
  if (w.p) retired.push_back(w.p);
  CAPGEN_HIP(hipMalloc(&w.p, bytes));
  w.bytes = bytes;
}
Workspace get_ws(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_ws.find(s);
  return it == g_ws.end() ? Workspace{} : it->second;
}

template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int ST, int KG = 1>
static void launch_cfg(const GemmArgs& g, hipStream_t s, int splitk) {
  require(KG == 1 || splitk == 1, "gemm: k-group variants run without grid split-K");
  const int tn = (g.N + BN - 1) / BN, tm = (g.M + BM - 1) / BM;
  const int nblk = tn * tm * splitk;
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  float* ws = nullptr;
  int* cnt = nullptr;
  if (splitk > 1) {
    const size_t bytes = (size_t)tn * tm * splitk * BM * BN * sizeof(float);
    const Workspace w = get_ws(s);
    require(w.bytes >= bytes && w.cnt, "gemm: split-K workspace too small (tune outside capture)");
    require(tn * tm <= kMaxTiles, "gemm: too many tiles for split-K");
    ws = w.p, cnt = w.cnt;
    if (g_splitk_proto & 32) {  // diagnostic: rotate over 4 ticket arrays (kMaxTiles / 4 each)
      static std::map<hipStream_t, int> rot;
      cnt += (rot[s]++ & 3) * (kMaxTiles / 4);
      require(tn * tm <= kMaxTiles / 4, "gemm: too many tiles for ticket rotation");
    }
    // tickets: zeroed once at allocation and re-armed by each tile's last arriver (an atomic
    // exchange, gemm_tile); a per-launch memset (the guide's 'Re-initialise every call') costs
    // 6-40 us per launch as a separate node on ROCm 7 (tools/splitk_stress.py time) -- diagnostic
    // bit 8 of capgen_debug_splitk_protocol restores it
    if (g_splitk_proto & 8) CAPGEN_HIP(hipMemsetAsync(cnt, 0, (size_t)(tn * tm + 3) / 4 * 16, s));
  }
  // group_m ~ sqrt(tiles per XCD), so each XCD's tile block is about square
  static const bool grouping = [] {
    const char* e = std::getenv("CAPGEN_GEMM_GROUP");
    return !(e && e[0] == '0');
  }();
  int group_m = 0;
  if (grouping) {
    const double per_xcd = (double)tn * tm / 8.0;
    group_m = std::max(1, std::min(tm, (int)std::lround(std::sqrt(per_xcd))));
  }
  GemmArgs gk = g;
  if ((g_splitk_proto & 4096) && g_timing_buf) gk.stamp = g_timing_buf;  // (ablation build: phase timing)
  gemm_bf16_kernel<TO, TA, TB, BM, BN, WM, WN, ST, KG>
      <<<nblk, 64 * WM * WN * KG, 0, s>>>(gk, tn, nblk, g_zero_page[dev], splitk, ws, cnt, group_m, g_splitk_proto & ~8);
}

// split-K workspace bound for any variant (tiles up to 256x128)
size_t splitk_bytes(const GemmArgs& g, int splitk) {
  return (size_t)((g.M + 255) / 256 * 256) * ((g.N + 127) / 128 * 128) * splitk * sizeof(float);
}

int g_variant = 0;  // experiment selector (capgen_debug_gemm_variant); 0 = tuned/heuristic

// Tile / wave-grid / pipeline-depth variants.  Every variant accumulates the same K tiles
// in the same order with the same MFMA sequence, so results are bit-identical across
// variants: the choice is a pure speed decision (made per shape by the autotuner).
constexpr int NVARIANTS = 30;
const char* kVariantName[NVARIANTS + 1] = {"auto",        "128x128w4s3", "128x128w8s2",  "128x128w4s2",
                                           "128x64w4s2",  "64x128w4s2",  "64x64w4s2",    "64x64w4s3",
                                           "128x64w8s2",  "256x128w16s2", "128x128w16s2", "256x64w8s2",
                                           "64x64w4s4",   "64x64w4s6",   "128x64w4s4",   "64x128w4s4",
                                           "128x128w4s4", "32x64w4s2",   "64x32w4s2",    "32x32w4s2",
                                           "64x64w8s2",   "32x64w4s3",   "64x32w4s3",
                                           // k-group variants (TileCfg KG): 'k2' = 2 k-groups of the waves named
                                           "64x64w4k2s2", "64x64w4k2s3", "32x64w4k2s3", "64x64w4k4s2",
                                           "32x64w4k4s2", "128x64w4k2s2", "64x128w4k2s2", "32x64w4k2s2"};

// output tile width (columns) of each variant
constexpr int kVariantBN[NVARIANTS + 1] = {0,  128, 128, 128, 64, 128, 64, 64, 64, 128, 128, 64,
                                           64, 64,  64,  128, 128, 64, 32, 32, 64, 64,  32,
                                           64, 64,  64,  64,  64,  64, 128, 64};
// k-groups of each variant (grid split-K only for KG == 1)
constexpr int kVariantKG[NVARIANTS + 1] = {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                           1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 4, 4, 2, 2, 2};

// A tile whose output row segment is narrower than a 128-B cache line shares lines of C with
// its neighbour tile, which another workgroup -- possibly on another XCD -- writes in the same
// launch.  With a read-modify-write epilogue (beta: C is read first) each XCD's L2 then holds
// the whole line with the neighbour's half stale, and a later kernel on that XCD can read the
// stale half (measured: ~1 in 5 bf16 c2s backward passes differed run to run in the encoder
// gradients, tools/bwd_bisect.py).  Such variants are never chosen, so every line of C is
// written by exactly one workgroup.  CAPGEN_ALLOW_PARTIAL_LINES=1 lifts the rule (diagnostic).
template <typename TO>
static bool whole_lines(int v) {
  static const bool allow = [] {
    const char* e = std::getenv("CAPGEN_ALLOW_PARTIAL_LINES");
    return e && e[0] == '1';
  }();
  return allow || kVariantBN[v] * (int)sizeof(TO) >= 128;
}

template <typename TO, bool TA, bool TB>
static void launch_variant(int v, const GemmArgs& g, hipStream_t s, int sk = 1) {
  switch (v) {
    case 1: return launch_cfg<TO, TA, TB, 128, 128, 2, 2, 3>(g, s, sk);
    case 2: return launch_cfg<TO, TA, TB, 128, 128, 2, 4, 2>(g, s, sk);
    case 3: return launch_cfg<TO, TA, TB, 128, 128, 2, 2, 2>(g, s, sk);
    case 4: return launch_cfg<TO, TA, TB, 128, 64, 2, 2, 2>(g, s, sk);
    case 5: return launch_cfg<TO, TA, TB, 64, 128, 2, 2, 2>(g, s, sk);
    case 6: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 2>(g, s, sk);
    case 7: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 3>(g, s, sk);
    case 8: return launch_cfg<TO, TA, TB, 128, 64, 4, 2, 2>(g, s, sk);
    case 9: return launch_cfg<TO, TA, TB, 256, 128, 4, 4, 2>(g, s, sk);
    case 10: return launch_cfg<TO, TA, TB, 128, 128, 4, 4, 2>(g, s, sk);
    case 11: return launch_cfg<TO, TA, TB, 256, 64, 4, 2, 2>(g, s, sk);
    case 12: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 4>(g, s, sk);
    case 13: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 6>(g, s, sk);
    case 14: return launch_cfg<TO, TA, TB, 128, 64, 2, 2, 4>(g, s, sk);
    case 15: return launch_cfg<TO, TA, TB, 64, 128, 2, 2, 4>(g, s, sk);
    case 16: return launch_cfg<TO, TA, TB, 128, 128, 2, 2, 4>(g, s, sk);
    // small tiles: more workgroups per CU for the latency-bound small GEMMs of the step
    case 17: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 2>(g, s, sk);
    case 18: return launch_cfg<TO, TA, TB, 64, 32, 2, 2, 2>(g, s, sk);
    case 19: return launch_cfg<TO, TA, TB, 32, 32, 2, 2, 2>(g, s, sk);
    case 20: return launch_cfg<TO, TA, TB, 64, 64, 4, 2, 2>(g, s, sk);
    case 21: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 3>(g, s, sk);
    case 22: return launch_cfg<TO, TA, TB, 64, 32, 2, 2, 3>(g, s, sk);
    case 23: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 2, 2>(g, s, sk);
    case 24: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 3, 2>(g, s, sk);
    case 25: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 3, 2>(g, s, sk);
    case 26: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 2, 4>(g, s, sk);
    case 27: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 2, 4>(g, s, sk);
    case 28: return launch_cfg<TO, TA, TB, 128, 64, 2, 2, 2, 2>(g, s, sk);
    case 29: return launch_cfg<TO, TA, TB, 64, 128, 2, 2, 2, 2>(g, s, sk);
    case 30: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 2, 2>(g, s, sk);
    default: throw Error("gemm: unknown variant");
  }
}

int heuristic_variant(const GemmArgs& g) {
  const long b64 = (long)((g.M + 63) / 64) * ((g.N + 63) / 64);
  return b64 <= 4096 ? 6 : 3;
}

struct TuneKey {
  int M, N, K, ta, tb, out;
  bool operator<(const TuneKey& o) const {
    return std::tie(M, N, K, ta, tb, out) < std::tie(o.M, o.N, o.K, o.ta, o.tb, o.out);
  }
};
struct Choice {
  int variant, splitk;
};
std::map<TuneKey, Choice> g_tuned;
std::mutex g_tune_mu;
int g_live_tuned = 0;  // shapes (plain + grouped) tuned live in this process

bool autotune_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("CAPGEN_AUTOTUNE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Tuning-time clock of one (variant, split-K) candidate: 3 launches.  In the step every GEMM
// reads operands that are not in this XCD's L2 (the A operand was just written by the previous
// kernel -- possibly on another XCD -- and the weights were last touched a step ago), so the
// latency-bound small shapes run ~2x their L2-warm repeat time there (dec W2 1216x512x2048:
// 24.6 us in the step, 11.9 us repeated).  With CAPGEN_TUNE_COLD (default on) each timed launch
// follows a 64 MB scrub write that evicts the L2s, so the tuner ranks candidates under the
// step's cache state; the scrub itself is outside the timed span.
static bool tune_cold() {
  static const bool on = [] {
    const char* e = std::getenv("CAPGEN_TUNE_COLD");
    return !(e && e[0] == '0');
  }();
  return on;
}
// CAPGEN_TUNE_BG=1 (experiment): each timed candidate runs beside a background stream kernel
// shaped like the step's bucket Adam (one 256-thread workgroup per CU streaming 96 MB read +
// write), so the ranking sees the contention the step's critical GEMMs run under
__global__ void tune_bg_kernel(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = a[i];
    v.x += 1.f;
    b[i] = v;
  }
}
static bool tune_bg() {
  static const bool on = [] {
    const char* e = std::getenv("CAPGEN_TUNE_BG");
    return e && e[0] == '1';
  }();
  return on;
}
static void tune_bg_launch(hipStream_t s) {
  static hipStream_t bg = nullptr;
  static float4* buf = nullptr;
  constexpr size_t kN = (48u << 20) / 16;  // 48 MB in, 48 MB out
  if (!bg) {
    CAPGEN_HIP(hipStreamCreateWithFlags(&bg, hipStreamNonBlocking));
    CAPGEN_HIP(hipMalloc(&buf, 2 * kN * sizeof(float4)));
    CAPGEN_HIP(hipMemset(buf, 0, 2 * kN * sizeof(float4)));
    CAPGEN_HIP(hipDeviceSynchronize());
  }
  CAPGEN_HIP(hipStreamSynchronize(s));  // the scrub is done: background and candidate start together
  tune_bg_kernel<<<256, 256, 0, bg>>>(buf, buf + kN, kN);
}
static void tune_bg_wait() {
  CAPGEN_HIP(hipDeviceSynchronize());
}

template <typename F>
static float tune_time(F&& launch, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  launch();  // warm-up (code, TLB)
  if (!tune_cold()) {
    CAPGEN_HIP(hipEventRecord(e0, s));
    for (int r = 0; r < 3; ++r) launch();
    CAPGEN_HIP(hipEventRecord(e1, s));
    CAPGEN_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    CAPGEN_HIP(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  }
  static std::map<int, void*> scrub;  // per device, never freed (tuning-time helper)
  constexpr size_t kScrub = 64u << 20;
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  void*& buf = scrub[dev];
  if (!buf) CAPGEN_HIP(hipMalloc(&buf, kScrub));
  float tot = 0.f;
  for (int r = 0; r < 3; ++r) {
    CAPGEN_HIP(hipMemsetAsync(buf, r, kScrub, s));
    if (tune_bg()) tune_bg_launch(s);
    CAPGEN_HIP(hipEventRecord(e0, s));
    launch();
    CAPGEN_HIP(hipEventRecord(e1, s));
    CAPGEN_HIP(hipEventSynchronize(e1));
    if (tune_bg()) tune_bg_wait();
    float ms = 0.f;
    CAPGEN_HIP(hipEventElapsedTime(&ms, e0, e1));
    tot += ms;
  }
  return tot;
}

template <typename TO, bool TA, bool TB>
static Choice tune(const GemmArgs& g, hipStream_t s) {
  // time every (variant, split-K) on a scratch output (inputs untouched, beta forced to 0)
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  GemmArgs t = g;
  void* scratch = nullptr;
  if (t.C2) t.C2 = nullptr, t.nsplit = 0, t.ldc = std::max<int64_t>(t.ldc, t.N);  // all columns to scratch
  CAPGEN_HIP(hipMalloc(&scratch, (size_t)t.M * t.ldc * sizeof(TO)));
  t.C = scratch;
  t.beta = 0;
  t.colsum = nullptr;
  t.stamp = nullptr;
  hipEvent_t e0, e1;
  CAPGEN_HIP(hipEventCreate(&e0));
  CAPGEN_HIP(hipEventCreate(&e1));
  Choice best{heuristic_variant(g), 1};
  float best_ms = 1e30f;
  const int nk = (g.K + BK - 1) / BK;
  // split-K factor cap (CAPGEN_MAX_SPLITK, default 8).  Round 1 capped it at 2 because the bf16
  // step was not reproducible run to run with higher factors; the causes were a sub-line output
  // tile under a read-modify-write epilogue (whole_lines) and the combine's ticket re-arm /
  // missing acquire (gemm_tile) -- tools/step_det_probe.py: 0 of 60 diverging runs at cap 8 now.
  static const int max_sk = [] {
    const char* e = std::getenv("CAPGEN_MAX_SPLITK");
    return e ? std::max(1, std::atoi(e)) : 8;
  }();
  // diagnostic: CAPGEN_SPLITK_K=k1,k2,... allows split-K only for those K (bisecting a step)
  static const std::vector<int> sk_only = [] {
    std::vector<int> v;
    if (const char* e = std::getenv("CAPGEN_SPLITK_K"))
      for (const char* p = e; *p;) {
        v.push_back(std::atoi(p));
        while (*p && *p != ',') ++p;
        if (*p) ++p;
      }
    return v;
  }();
  const bool sk_ok = sk_only.empty() || std::find(sk_only.begin(), sk_only.end(), g.K) != sk_only.end();
  for (int sk : {1, 2, 3, 4, 6, 8}) {
    if (sk > max_sk || (sk > 1 && (nk < 4 * sk || !sk_ok))) break;
    if (sk > 1) ensure_ws(s, splitk_bytes(g, sk));
    for (int v = 1; v <= NVARIANTS; ++v) {
      if (!whole_lines<TO>(v) || (sk > 1 && kVariantKG[v] > 1)) continue;
      const float ms = tune_time([&] { launch_variant<TO, TA, TB>(v, t, s, sk); }, s, e0, e1);
      if (ms < best_ms) best_ms = ms, best = Choice{v, sk};
    }
  }
  CAPGEN_HIP(hipEventDestroy(e0));
  CAPGEN_HIP(hipEventDestroy(e1));
  CAPGEN_HIP(hipFree(scratch));
  if (std::getenv("CAPGEN_AUTOTUNE_LOG"))
    std::fprintf(stderr, "[capgen gemm] M=%d N=%d K=%d ta=%d tb=%d out=%s -> %s splitk=%d (%.2f us)\n", g.M, g.N, g.K,
                 TA, TB, sizeof(TO) == 4 ? "f32" : "bf16", kVariantName[best.variant], best.splitk,
                 best_ms * 1e3f / 3);
  return best;
}

template <typename TO, bool TA, bool TB>
static void launch_bf16_tiles(const GemmArgs& g, hipStream_t s) {
  Choice c{g_variant % 100, std::max(1, g_variant / 100)};  // forced: variant + 100 * splitk
  if (TA && c.variant == 0) {  // experiment knob: weight-gradient (TN) GEMMs on a fixed variant
    static const int dwv = [] {
      const char* e = std::getenv("CAPGEN_DW_VARIANT");
      return e ? std::atoi(e) : 0;
    }();
    if (dwv) c = Choice{dwv % 100, std::max(1, dwv / 100)};
  }
  // experiment knob: CAPGEN_GEMM_FORCE="M,N,K,ta,tb,v[;...]" pins one shape's choice (variant v +
  // 100 * split-K), e.g. to A/B a critical-path GEMM in the step rather than alone
  static const std::map<TuneKey, int> forced = [] {
    std::map<TuneKey, int> m;
    if (const char* e = std::getenv("CAPGEN_GEMM_FORCE")) {
      int M, N, K, ta, tb, v, n = 0;
      for (const char* p = e; *p;) {
        if (std::sscanf(p, "%d,%d,%d,%d,%d,%d%n", &M, &N, &K, &ta, &tb, &v, &n) != 6) break;
        m[TuneKey{M, N, K, ta, tb, 2}] = v, m[TuneKey{M, N, K, ta, tb, 4}] = v;
        p += n;
        if (*p == ';') ++p;
      }
    }
    return m;
  }();
  if (c.variant == 0 && !forced.empty()) {
    auto it = forced.find(TuneKey{g.M, g.N, g.K, TA, TB, (int)sizeof(TO)});
    if (it != forced.end()) c = Choice{it->second % 100, std::max(1, it->second / 100)};
  }
  if (c.splitk > 1) ensure_ws(s, splitk_bytes(g, c.splitk));
  if (c.variant == 0) {
    c.variant = heuristic_variant(g);
    TuneKey key{g.M, g.N, g.K, TA, TB, (int)sizeof(TO)};
    std::lock_guard<std::mutex> lk(g_tune_mu);
    auto it = g_tuned.find(key);  // tuned in this process or loaded from the persisted table
    if (it != g_tuned.end()) {
      c = it->second;
    } else if (autotune_enabled()) {
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      CAPGEN_HIP(hipStreamIsCapturing(s, &st));
      if (st == hipStreamCaptureStatusNone) {
        // a shape the table does not hold: tune it on an idle device (every stream drained, so
        // no concurrent kernel shares the CUs or the caches with the candidates' clock, and the
        // candidates run strictly between the work issued before and after this call)
        CAPGEN_HIP(hipDeviceSynchronize());
        c = g_tuned[key] = tune<TO, TA, TB>(g, s);
        CAPGEN_HIP(hipStreamSynchronize(s));
        ++g_live_tuned;
      }
    }
  }
  if (c.splitk > 1) {
    const size_t bytes = splitk_bytes(g, c.splitk);
    const Workspace w = get_ws(s);
    if (!(w.cnt && w.bytes >= bytes)) {  // (the common case skips the capture query: host time)
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      CAPGEN_HIP(hipStreamIsCapturing(s, &st));
      if (st == hipStreamCaptureStatusNone) ensure_ws(s, bytes);
      else c.splitk = 1;  // no allocation inside a capture
    }
  }
  launch_variant<TO, TA, TB>(c.variant, g, s, c.splitk);
}

template <typename TO>
static void launch_bf16_layout(const GemmArgs& g, bool ta, bool tb, hipStream_t s) {
  if (!ta && !tb) launch_bf16_tiles<TO, false, false>(g, s);
  else if (!ta && tb) launch_bf16_tiles<TO, false, true>(g, s);
  else if (ta && !tb) launch_bf16_tiles<TO, true, false>(g, s);
  else launch_bf16_tiles<TO, true, true>(g, s);
}

// ---- grouped launch ---------------------------------------------------------------------
template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int ST>
static void launch_group_cfg(const GemmArgs* ps, int n, hipStream_t s) {
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  GemmGroup gg;
  gg.n = n;
  int tot = 0;
  for (int i = 0; i < n; ++i) {
    const int tn = (ps[i].N + BN - 1) / BN, tm = (ps[i].M + BM - 1) / BM;
    gg.start[i] = tot, gg.tiles_n[i] = tn, gg.p[i] = ps[i];
    tot += tn * tm;
  }
  gg.start[n] = tot;
  // the grouped (weight-gradient) grid is capped at one workgroup per CU, each looping over its
  // tiles: the side-stream dW work then leaves room on every CU for the critical stream's
  // latency-bound kernels (step 3.44-3.47 vs 3.54 ms uncapped; 64 workgroups: 3.75 ms, the dW
  // work becomes critical).  CAPGEN_DW_GRID overrides (0 = uncapped).
  static const int cap = [] {
    const char* e = std::getenv("CAPGEN_DW_GRID");
    if (e) return std::atoi(e) / 8 * 8;
    int n = 0, dev = 0;
    CAPGEN_HIP(hipGetDevice(&dev));
    CAPGEN_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    return std::max(8, n / 8 * 8);
  }();
  const int G = cap > 0 ? std::min(tot, cap) : tot;
  gemm_bf16_grouped_kernel<TO, TA, TB, BM, BN, WM, WN, ST><<<G, 64 * WM * WN, 0, s>>>(gg, tot, G, g_zero_page[dev]);
}

// the variants worth a grouped launch (many tiles already: no split-K)
constexpr int kGroupVariants[] = {6, 20, 17, 18, 19, 4, 8, 1, 3, 10};

template <typename TO, bool TA, bool TB>
static void launch_group_variant(int v, const GemmArgs* ps, int n, hipStream_t s) {
  switch (v) {
    case 1: return launch_group_cfg<TO, TA, TB, 128, 128, 2, 2, 3>(ps, n, s);
    case 3: return launch_group_cfg<TO, TA, TB, 128, 128, 2, 2, 2>(ps, n, s);
    case 4: return launch_group_cfg<TO, TA, TB, 128, 64, 2, 2, 2>(ps, n, s);
    case 6: return launch_group_cfg<TO, TA, TB, 64, 64, 2, 2, 2>(ps, n, s);
    case 8: return launch_group_cfg<TO, TA, TB, 128, 64, 4, 2, 2>(ps, n, s);
    case 10: return launch_group_cfg<TO, TA, TB, 128, 128, 4, 4, 2>(ps, n, s);
    case 17: return launch_group_cfg<TO, TA, TB, 32, 64, 2, 2, 2>(ps, n, s);
    case 18: return launch_group_cfg<TO, TA, TB, 64, 32, 2, 2, 2>(ps, n, s);
    case 19: return launch_group_cfg<TO, TA, TB, 32, 32, 2, 2, 2>(ps, n, s);
    case 20: return launch_group_cfg<TO, TA, TB, 64, 64, 4, 2, 2>(ps, n, s);
    default: throw Error("gemm_grouped: unknown variant");
  }
}

std::map<std::vector<int>, int> g_group_tuned;

template <typename TO, bool TA, bool TB>
static void launch_group(const GemmArgs* ps, int n, hipStream_t s) {
  std::vector<int> key{TA, TB, (int)sizeof(TO)};
  for (int i = 0; i < n; ++i) key.insert(key.end(), {ps[i].M, ps[i].N, ps[i].K});
  int v = g_variant % 100;
  static const int forced = [] {  // experiment knob: every grouped launch on one variant
    const char* e = std::getenv("CAPGEN_DWG_VARIANT");
    return e ? std::atoi(e) : 0;
  }();
  if (v == 0 && forced) v = forced;
  if (v == 0) {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    auto it = g_group_tuned.find(key);
    if (it != g_group_tuned.end()) {
      v = it->second;
    } else {
      v = kGroupVariants[0];
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      CAPGEN_HIP(hipStreamIsCapturing(s, &st));
      if (st == hipStreamCaptureStatusNone && autotune_enabled()) {
        CAPGEN_HIP(hipDeviceSynchronize());  // idle device (see launch_bf16_tiles)
        ++g_live_tuned;
        // time each variant on scratch outputs (inputs untouched, beta forced to 0)
        std::vector<GemmArgs> t(ps, ps + n);
        std::vector<void*> scratch(n);
        for (int i = 0; i < n; ++i) {
          CAPGEN_HIP(hipMalloc(&scratch[i], (size_t)t[i].M * t[i].ldc * sizeof(TO)));
          t[i].C = scratch[i], t[i].beta = 0, t[i].colsum = nullptr, t[i].stamp = nullptr;
        }
        hipEvent_t e0, e1;
        CAPGEN_HIP(hipEventCreate(&e0));
        CAPGEN_HIP(hipEventCreate(&e1));
        float best = 1e30f;
        for (int cand : kGroupVariants) {
          if (!whole_lines<TO>(cand)) continue;
          const float ms = tune_time([&] { launch_group_variant<TO, TA, TB>(cand, t.data(), n, s); }, s, e0, e1);
          if (ms < best) best = ms, v = cand;
        }
        CAPGEN_HIP(hipEventDestroy(e0));
        CAPGEN_HIP(hipEventDestroy(e1));
        for (void* p : scratch) CAPGEN_HIP(hipFree(p));
        CAPGEN_HIP(hipStreamSynchronize(s));
        g_group_tuned[key] = v;
        if (std::getenv("CAPGEN_AUTOTUNE_LOG"))
          std::fprintf(stderr, "[capgen gemm] group of %d (M=%d N=%d K=%d first) -> %s (%.2f us)\n", n, ps[0].M,
                       ps[0].N, ps[0].K, kVariantName[v], best * 1e3f / 3);
      }
    }
  }
  launch_group_variant<TO, TA, TB>(v, ps, n, s);
}

static void gemm_grouped_impl(const GemmArgs* ps, int n, DType out, bool ta, bool tb, hipStream_t s);
// CAPGEN_HOST_TIMING (diagnostic): average host time of a grouped launch, printed every 500 calls
void gemm_grouped(const GemmArgs* ps, int n, DType out, bool ta, bool tb, hipStream_t s) {
  static const bool timing = std::getenv("CAPGEN_HOST_TIMING") != nullptr;
  if (!timing) return gemm_grouped_impl(ps, n, out, ta, tb, s);
  static double tot = 0;
  static long cnt = 0;
  const auto t0 = std::chrono::steady_clock::now();
  gemm_grouped_impl(ps, n, out, ta, tb, s);
  tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  if (++cnt % 500 == 0) {
    std::fprintf(stderr, "[capgen host] gemm_grouped() call: %.2f us average over 500\n", tot / 500);
    tot = 0;
  }
}
static void gemm_grouped_impl(const GemmArgs* ps, int n, DType out, bool ta, bool tb, hipStream_t s) {
  require(n >= 1 && n <= kMaxGroup, "gemm_grouped: 1..kMaxGroup problems");
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  require(g_zero_page[dev] != nullptr, "gemm: gemm_init() not called on this device");
  std::vector<GemmArgs> pw(ps, ps + n);  // write-through default, as gemm_bf16
  for (auto& g : pw) {
    if (g.wt < 0) g.wt = wt_default();
    if ((int64_t)g.M * g.ldc * (int64_t)dsize(out) >= (int64_t)0x7FFFFFFF) g.wt = 0;
  }
  ps = pw.data();
  for (int i = 0; i < n; ++i) {
    const GemmArgs& g = ps[i];
    require(g.M > 0 && g.N > 0 && g.K > 0 && g.N % 4 == 0 && g.ldc % 4 == 0 && (g.aux == nullptr || g.ldaux % 4 == 0),
            "gemm_grouped: bad problem shape");
    require(((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0, "gemm_grouped: operands must be 16-B aligned");
  }
  if (hz::active()) {
    std::vector<hz::Rgn> v;
    for (int i = 0; i < n; ++i) gemm_hz_regions(ps[i], DType::BF16, out, ta, tb, v);
    hz::op(s, "gemm grouped (dW)", v.data(), v.size());
  }
  if (out == DType::F32) {
    if (ta && tb) launch_group<float, true, true>(ps, n, s);
    else if (!ta && tb) launch_group<float, false, true>(ps, n, s);
    else throw Error("gemm_grouped: layout not instantiated");
  } else {
    if (!ta && tb) launch_group<bf16, false, true>(ps, n, s);
    else if (!ta && !tb) launch_group<bf16, false, false>(ps, n, s);
    else throw Error("gemm_grouped: layout not instantiated");
  }
  CAPGEN_HIP(hipGetLastError());
}

// ---- persisted autotune table --------------------------------------------------------------
// Text, one choice per line:  g M N K ta tb out_bytes variant splitk
//                             G ta tb out_bytes n M1 N1 K1 ... Mn Nn Kn variant
int gemm_tune_load(const char* path) {
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  std::lock_guard<std::mutex> lk(g_tune_mu);
  int n = 0;
  char line[1024];
  while (std::fgets(line, sizeof line, f)) {
    if (line[0] == 'g') {
      TuneKey k{};
      Choice c{};
      if (std::sscanf(line + 1, "%d %d %d %d %d %d %d %d", &k.M, &k.N, &k.K, &k.ta, &k.tb, &k.out, &c.variant,
                      &c.splitk) == 8 &&
          c.variant >= 1 && c.variant <= NVARIANTS && c.splitk >= 1 && c.splitk <= 16) {
        g_tuned.emplace(k, c);
        ++n;
      }
    } else if (line[0] == 'G') {
      std::vector<int> v;
      const char* p = line + 1;
      int x, used = 0;
      while (std::sscanf(p, "%d%n", &x, &used) == 1) v.push_back(x), p += used;
      if (v.size() >= 5 && v.size() == 4 + 3 * (size_t)v[3] + 1) {
        const int var = v.back();
        std::vector<int> key{v[0], v[1], v[2]};
        key.insert(key.end(), v.begin() + 4, v.end() - 1);
        g_group_tuned.emplace(key, var);
        ++n;
      }
    }
  }
  std::fclose(f);
  return n;
}

int gemm_tune_save(const char* path) {
  FILE* f = std::fopen(path, "w");
  if (!f) return -1;
  std::lock_guard<std::mutex> lk(g_tune_mu);
  std::fprintf(f, "# capgen bf16 GEMM autotune table (gfx950): g M N K ta tb out_bytes variant splitk | "
                  "G ta tb out_bytes n (M N K)xn variant\n");
  int n = 0;
  for (auto& kv : g_tuned) {
    const TuneKey& k = kv.first;
    std::fprintf(f, "g %d %d %d %d %d %d %d %d  # %s\n", k.M, k.N, k.K, k.ta, k.tb, k.out, kv.second.variant,
                 kv.second.splitk, kVariantName[kv.second.variant]);
    ++n;
  }
  for (auto& kv : g_group_tuned) {
    const std::vector<int>& k = kv.first;
    std::fprintf(f, "G %d %d %d %d", k[0], k[1], k[2], (int)(k.size() - 3) / 3);
    for (size_t i = 3; i < k.size(); ++i) std::fprintf(f, " %d", k[i]);
    std::fprintf(f, " %d  # %s\n", kv.second, kVariantName[kv.second]);
    ++n;
  }
  std::fclose(f);
  return n;
}

int gemm_tune_live_count() { return g_live_tuned; }

void gemm_set_variant(int v) { g_variant = v; }
void gemm_set_splitk_protocol(int p) { g_splitk_proto = p; }
void gemm_set_timing_buf(uint64_t* p) { g_timing_buf = p; }
void gemm_splitk_diag(int* out4, bool reset) {
  CAPGEN_HIP(hipDeviceSynchronize());
  CAPGEN_HIP(hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_sk_diag), 4 * sizeof(int)));
  if (reset) {
    const int z[4] = {0, 0, 0, 0};
    CAPGEN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sk_diag), z, sizeof(z)));
  }
}

// the persisted autotune table: $CAPGEN_TUNE_TABLE, else tune_gfx950.txt next to libcapgen.so
// ("0" or "": none), loaded once per process before the first GEMM
static void load_default_tune_table() {
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("CAPGEN_TUNE_TABLE");
    std::string path;
    if (e) {
      if (!e[0] || (e[0] == '0' && !e[1])) return;
      path = e;
    } else {
      Dl_info info;
      if (!dladdr((void*)&gemm_init, &info) || !info.dli_fname) return;
      path = info.dli_fname;
      const size_t slash = path.rfind('/');
      path = (slash == std::string::npos ? std::string(".") : path.substr(0, slash)) + "/tune_gfx950.txt";
    }
    const int n = gemm_tune_load(path.c_str());
    if (std::getenv("CAPGEN_AUTOTUNE_LOG")) std::fprintf(stderr, "[capgen gemm] tune table %s: %d entries\n", path.c_str(), n);
  });
}

void gemm_init() {
  load_default_tune_table();
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  require(dev >= 0 && dev < 64, "gemm_init: device index out of range");
  if (!g_zero_page[dev]) {
    CAPGEN_HIP(hipMalloc(&g_zero_page[dev], 4096));
    CAPGEN_HIP(hipMemset(g_zero_page[dev], 0, 4096));
    CAPGEN_HIP(hipDeviceSynchronize());  // ordered before work on non-blocking streams
  }
}

void gemm_bf16(const GemmArgs& g_in, DType out, bool ta, bool tb, hipStream_t s) {
  GemmArgs g = g_in;
  if (g.wt < 0) g.wt = wt_default();
  if ((int64_t)g.M * g.ldc * (int64_t)dsize(out) >= (int64_t)0x7FFFFFFF) g.wt = 0;  // (32-bit buffer offsets)
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  require(g_zero_page[dev] != nullptr, "gemm: gemm_init() not called on this device");
  require(g.N % 4 == 0 && g.ldc % 4 == 0 && (g.aux == nullptr || g.ldaux % 4 == 0),
          "gemm(bf16): N/ldc must be multiples of 4");
  // read-modify-write epilogue: every 128-B line of C must belong to one tile (whole_lines)
  require(!g.beta || (((uintptr_t)g.C & 127) == 0 && (g.ldc * (int64_t)dsize(out)) % 128 == 0),
          "gemm(bf16): beta=1 needs C rows 128-B aligned (one writer per cache line)");
  require(!g.ce_stats || (out == DType::BF16 && !ta && !tb && !g.beta && !g.C2 && !g.aux && !g.relu && !g.colsum &&
                          !g.cin && g.ce_tgt && g.ce_tlogit && g.ce_ld >= (g.N + 15) / 16),
          "gemm(bf16): the fused cross-entropy epilogue is a plain bf16 NT GEMM (+bias)");
  if (out == DType::F32) launch_bf16_layout<float>(g, ta, tb, s);
  else launch_bf16_layout<bf16>(g, ta, tb, s);
}

}  // namespace capgen
