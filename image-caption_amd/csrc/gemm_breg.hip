// capgen — bf16 GEMM with the B operand streamed into registers from a tiled copy (round 5).
//
// C[M,N] = A[M,K] . B[K,N] where B is handed over as its MFMA fragments: piece (j, ks) is 512 bf16,
// lane l holding B[32 ks + 8 (l >> 4) + e][16 j + (l & 15)], e = 0..7 -- the B fragment of
// v_mfma_f32_16x16x32_bf16 for column block j and 32-deep k-step ks, one coalesced 1-KB load
// (gemm_tile_b builds it from B stored [N][K] (nn.Linear weights, the forward) or [K][N]).
//
// The form of the attention fronts (qkv_attn.hip), measured against the LDS-DMA ring of gemm_tile.h
// by tools/breg_probe.hip (kernel durations under rocprofv3, `profiles/r05_breg_probe.txt`): the
// 4 waves of a workgroup split N, so each wave's weight fragments are private to it and go straight
// from L2 into a double-buffered register batch of QB k-steps; only the A rows (shared by the waves)
// pass through LDS -- a 2-stage ring filled from registers AD k-tiles ahead (plain loads and
// ds_write_b128: every wait is hipcc's own).  No ring DMA issue, no per-k-tile B fragment reads: at
// the decode step's shapes (M = 256 / 1280 rows, K = 512) 27-38 % below the ring's kernel time,
// 6-12 % at K = 2048.
//
// Tile: BM x BN, wave w = all BM rows x columns [w BN/4, (w+1) BN/4); A k-tiles of 32 KT; tiles are
// grouped per XCD (XCD x = blockIdx % 8 takes the x-th contiguous chunk of the M-major tile list:
// its tiles share A row panels).  The epilogue is gemm_tile.h's (bias, ReLU, ReLU' mask, beta, split
// output C2): lane holds C[m0 + 16 i + (l & 15)][n0 + w BN/4 + 16 f + 4 (l >> 4) + 0..3].
#include <type_traits>

#include "gemm_tile.h"
#include "hazard.h"

namespace capgen {
namespace {

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

template <typename TO, int BM, int BN, int QB, int AD, int KT>
__global__ void __launch_bounds__(256) breg_kernel(GemmArgs g) {
  constexpr int FM = BM / 16, WN = BN / 4, FN = WN / 16;
  constexpr int TPB = QB / KT;            // k-tiles per B batch
  constexpr int CPT = BM * KT * 4 / 256;  // 16-B A chunks per thread per k-tile
  constexpr int RB = KT * 64;             // LDS bytes per A row per stage
  static_assert(TPB % AD == 0 && AD % 2 == 0 && CPT >= 1 && FN >= 1, "breg tile shape");
  __shared__ __attribute__((aligned(16))) char sA[2][BM * RB];
  StampScope stamp_scope(g.stamp);
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = g.M, N = g.N, K = g.K;
  const int MT = (M + BM - 1) / BM, NT = N / BN, T = MT * NT;
  const int per = (T + 7) / 8;
  const int tile = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (tile >= T) return;
  const int mt = tile / NT, nt = tile % NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk = K / (32 * KT), nb = K / (32 * QB), KS = K / 32;
  const bf16* __restrict__ A = reinterpret_cast<const bf16*>(g.A);
  const bf16* __restrict__ Bt = reinterpret_cast<const bf16*>(g.bt);

  const bf16* brow[FN];
#pragma unroll
  for (int f = 0; f < FN; ++f) brow[f] = Bt + ((int64_t)((n0 + w * WN) / 16 + f) * KS * 64 + lane) * 8;
  bf16x8 bq[2][QB][FN];
  auto loadB = [&](int b, bf16x8 (&dst)[QB][FN]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < QB; ++q)
#pragma unroll
      for (int f = 0; f < FN; ++f) dst[q][f] = *reinterpret_cast<const bf16x8*>(brow[f] + (int64_t)(b * QB + q) * 512);
  };
  // A rows past M read row M - 1 (their results are never stored).  Gathered rows: the selection
  // kernels only produce ids in [0, V); the clamp keeps a foreign id inside the table (gemm.hip
  // requires a_table_rows > 0 for every gathered launch)
  const bf16* arow[CPT];
  int aoff[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int id = tid + 256 * c, row = id / (KT * 4), ch = id % (KT * 4);
    const int m = min(m0 + row, M - 1);
    const int ar_ = g.a_ids ? min(max(g.a_ids[(int64_t)m * g.a_ids_ld], 0), g.a_table_rows - 1) : m;
    arow[c] = A + (int64_t)ar_ * g.lda + ch * 8;
    aoff[c] = row * RB + ((ch ^ (row & 7)) * 16);
  }
  u32x4 ar[AD][CPT];  // A(t) in ar[t % AD], loaded AD - 1 k-tiles before its LDS write
  auto loadA = [&](int kt, u32x4 (&r)[CPT]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) r[c] = *reinterpret_cast<const u32x4*>(arow[c] + kt * KT * 32);
  };
  auto writeA = [&](int st, const u32x4 (&r)[CPT]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) *reinterpret_cast<u32x4*>(sA[st] + aoff[c]) = r[c];
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int f = 0; f < FN; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int i = 0; i < AD; ++i)
    if (i < nk) loadA(i, ar[i]);
  loadB(0, bq[0]);
  if (nb > 1) loadB(1, bq[1]);
  writeA(0, ar[0]);
  if (AD < nk) loadA(AD, ar[0]);

  // one B batch (TPB k-tiles) from register buffer H (a compile-time index: a runtime one sends the
  // batches to scratch)
  auto batch = [&](int b, auto Hc) __attribute__((always_inline)) {
    constexpr int H = decltype(Hc)::value;
#pragma unroll
    for (int tt = 0; tt < TPB; ++tt) {
      const int t = b * TPB + tt;  // t % AD == tt % AD: TPB is a multiple of AD
      __syncthreads();             // A(t) visible in stage t & 1; stage (t + 1) & 1 free
      if (t + 1 < nk) {
        writeA((tt + 1) & 1, ar[(tt + 1) % AD]);
        if (t + 1 + AD < nk) loadA(t + 1 + AD, ar[(tt + 1) % AD]);
      }
      const char* st = sA[tt & 1];
#pragma unroll
      for (int ks = 0; ks < KT; ++ks) {
        bf16x8 af[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = 16 * i + (lane & 15), ch = 4 * ks + (lane >> 4);
          af[i] = *reinterpret_cast<const bf16x8*>(st + row * RB + ((ch ^ (row & 7)) * 16));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int f = 0; f < FN; ++f)
            acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[H][KT * tt + ks][f], af[i], acc[i][f], 0, 0, 0);
      }
    }
    if (b + 2 < nb) loadB(b + 2, bq[H]);
  };
  for (int bb = 0; bb < nb; bb += 2) {
    batch(bb, std::integral_constant<int, 0>{});
    if (bb + 1 < nb) batch(bb + 1, std::integral_constant<int, 1>{});
  }
  const float alpha = g.alpha_ptr ? g.alpha * *g.alpha_ptr : g.alpha;
  tile_epilogue<TO, FM, FN, BM, WN>(g, acc, m0, n0, 0, w, lane, alpha, 0, 1);
}

// The LayerNorm of the decode step folded into its consumer (GemmArgs::ln_gamma; K = 512 = d): the
// LayerNorm input is v = A + ln_res (the producing Linear's output, bias included, and the residual),
// so a BM-row tile's whole A block (BM KB) is loaded once with its residual, normalised in registers
// and left in LDS for all 16 k-steps -- the separate LayerNorm launch and its dependent boundary go
// away.  Half-wave h of wave w owns rows 2 w + h + 8 i (i < BM / 8); its lane c holds columns
// 16 c .. 16 c + 15 of each, so the row statistics are 5 xor-shuffles.  The workgroups of column tile
// 0 also store y (the next producer's residual).  B as in breg_kernel: 16 k-steps in two register
// batches of 8, both issued before the A block.
constexpr float kLnEps = 1e-6f;  // modules.py:57,105 (ops.hip LN_EPS)

template <typename TO, int BM>
__global__ void __launch_bounds__(256) breg_ln_kernel(GemmArgs g) {
  constexpr int BN = 64, QB = 8, KD = 512, KS = KD / 32, RB = KD * 2, RH = BM / 8;  // RH rows per half-wave
  constexpr int FM = BM / 16, WN = BN / 4;  // one 16-column fragment per wave
  __shared__ __attribute__((aligned(16))) char sA[BM * RB];
  StampScope stamp_scope(g.stamp);
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = g.M, N = g.N;
  const int MT = (M + BM - 1) / BM, NT = N / BN, T = MT * NT;
  const int per = (T + 7) / 8;
  const int tile = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (tile >= T) return;
  const int mt = tile / NT, nt = tile % NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const bf16* __restrict__ A = reinterpret_cast<const bf16*>(g.A);
  const bf16* brow = reinterpret_cast<const bf16*>(g.bt) + ((int64_t)((n0 + w * WN) / 16) * KS * 64 + lane) * 8;
  bf16x8 bq[2][QB];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int q = 0; q < QB; ++q) bq[b][q] = *reinterpret_cast<const bf16x8*>(brow + (int64_t)(b * QB + q) * 512);

  const int h = lane >> 5, c = lane & 31;
  // (an absent residual reads the A rows again and adds nothing: resw = 0)
  const bf16* __restrict__ Rs = g.ln_res ? reinterpret_cast<const bf16*>(g.ln_res) : A;
  const int64_t ldr = g.ln_res ? KD : g.lda;
  const float resw = g.ln_res ? 1.f : 0.f;
  u32x4 av[RH][2], rv[RH][2];
  int idv[RH];
#pragma unroll
  for (int i = 0; i < RH; ++i) {
    const int m = min(m0 + 2 * w + h + 8 * i, M - 1);
    const bf16* p = A + (int64_t)m * g.lda + 16 * c;
    const bf16* q = Rs + (int64_t)m * ldr + 16 * c;
    av[i][0] = *reinterpret_cast<const u32x4*>(p);
    av[i][1] = *reinterpret_cast<const u32x4*>(p + 8);
    rv[i][0] = *reinterpret_cast<const u32x4*>(q);
    rv[i][1] = *reinterpret_cast<const u32x4*>(q + 8);
    idv[i] = g.ln_ids ? g.ln_ids[(int64_t)m * g.ln_ids_ld] : 0;
  }
  float gm[16], bt[16];
#pragma unroll
  for (int e = 0; e < 16; e += 4) {
    const float4 g4 = *reinterpret_cast<const float4*>(g.ln_gamma + 16 * c + e);
    const float4 b4 = *reinterpret_cast<const float4*>(g.ln_beta + 16 * c + e);
    gm[e] = g4.x, gm[e + 1] = g4.y, gm[e + 2] = g4.z, gm[e + 3] = g4.w;
    bt[e] = b4.x, bt[e + 1] = b4.y, bt[e + 2] = b4.z, bt[e + 3] = b4.w;
  }
  bf16* __restrict__ Y = reinterpret_cast<bf16*>(g.ln_y);
#pragma unroll
  for (int i = 0; i < RH; ++i) {
    const int r = 2 * w + h + 8 * i;
    float x[16];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x[2 * e] = fmaf(resw, __uint_as_float(rv[i][e >> 2][e & 3] << 16), __uint_as_float(av[i][e >> 2][e & 3] << 16));
      x[2 * e + 1] = fmaf(resw, __uint_as_float(rv[i][e >> 2][e & 3] & 0xffff0000u),
                          __uint_as_float(av[i][e >> 2][e & 3] & 0xffff0000u));
    }
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) s += x[e];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)KD;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float t = x[e] - mean;
      q = fmaf(t, t, q);
    }
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o, 64);
    const float rstd = 1.0f / sqrtf(q / (float)KD + kLnEps);
    const float keep = g.ln_ids && idv[i] == g.ln_pad ? 0.f : 1.f;
    bf16x8 y[2];
#pragma unroll
    for (int e = 0; e < 16; ++e) y[e >> 3][e & 7] = (bf16)(((x[e] - mean) * rstd * gm[e] + bt[e]) * keep);
#pragma unroll
    for (int k = 0; k < 2; ++k) *reinterpret_cast<bf16x8*>(sA + r * RB + (((2 * c + k) ^ (r & 7)) * 16)) = y[k];
    if (nt == 0 && m0 + r < M) {
#pragma unroll
      for (int k = 0; k < 2; ++k) *reinterpret_cast<bf16x8*>(Y + (int64_t)(m0 + r) * KD + 16 * c + 8 * k) = y[k];
    }
  }
  __syncthreads();

  f32x4 acc[FM][1];
#pragma unroll
  for (int i = 0; i < FM; ++i) acc[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 af[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = 16 * i + (lane & 15), ch = 4 * ks + (lane >> 4);
      af[i] = *reinterpret_cast<const bf16x8*>(sA + row * RB + ((ch ^ (row & 7)) * 16));
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
      acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ks / QB][ks % QB], af[i], acc[i][0], 0, 0, 0);
  }
  const float alpha = g.alpha_ptr ? g.alpha * *g.alpha_ptr : g.alpha;
  tile_epilogue<TO, FM, 1, BM, WN>(g, acc, m0, n0, 0, w, lane, alpha, 0, 1);
}

// B[k][n] of B stored [N][K] (tb = 0) or [K][N] (tb = 1) -> the fragment pieces: one thread per
// (piece, lane) writes 16 B; the [N][K] form reads 16 contiguous bytes, the [K][N] form 8 strided bf16
__global__ void tile_b_kernel(const bf16* __restrict__ B, int64_t ldb, int tb, int N, int K, bf16* __restrict__ Bt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int KS = K / 32;
  if (i >= (int64_t)(N / 16) * KS * 64) return;
  const int lane = (int)(i & 63);
  const int64_t p = i >> 6;
  const int j = (int)(p / KS), ks = (int)(p % KS);
  const int n = 16 * j + (lane & 15), k0 = 32 * ks + 8 * (lane >> 4);
  bf16x8 v;
  if (tb) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = B[(int64_t)(k0 + e) * ldb + n];
  } else {
    v = *reinterpret_cast<const bf16x8*>(B + (int64_t)n * ldb + k0);
  }
  *reinterpret_cast<bf16x8*>(Bt + i * 8) = v;
}

template <typename TO, int BM, int BN, int QB, int AD, int KT>
void launch(const GemmArgs& g, hipStream_t s) {
  const int T = ((g.M + BM - 1) / BM) * (g.N / BN);
  breg_kernel<TO, BM, BN, QB, AD, KT><<<((T + 7) / 8) * 8, 256, 0, s>>>(g);
}

template <typename TO>
void launch_ln(const GemmArgs& g, hipStream_t s) {
  // 16-row tiles (greedy 8.73-8.75 vs 9.30-9.39 ms per C4 batch with 32-row ones; beam 5 folded with
  // 16-row tiles 13.56-13.57 vs 12.82-12.84 unfolded, so beam keeps the separate LayerNorms)
  const int T = ((g.M + 15) / 16) * (g.N / 64);
  breg_ln_kernel<TO, 16><<<((T + 7) / 8) * 8, 256, 0, s>>>(g);
}

}  // namespace

// the launch choice: 64 x 64 tiles with 4-step batches for wide outputs at >= 1024 rows
// (tools/breg_probe.hip, kernel durations), else 16 x 64 tiles, 128-deep k-tiles and 8-step batches --
// twice the workgroups of the probe's 32 x 64 choice, each with half the serial latency: C4 greedy
// 8.17-8.22 vs 8.61-8.70 ms, beam 5 12.64-12.70 vs 12.80-12.83 (in the decode, alternating libraries,
// profiles/r05_decode_16row_tiles.txt; 16-row tiles for the wide outputs too: beam 13.24-13.29)
static bool breg_wide(const GemmArgs& g) { return g.N >= 1536 && g.M >= 1024; }

bool gemm_breg_ok(const GemmArgs& g) {
  const int kq = breg_wide(g) ? 128 : 256;  // 32 * QB
  const bool ln_ok = !g.ln_gamma || (g.K == 512 && g.ln_beta && g.ln_y && g.ln_y != g.A && g.ln_y != g.ln_res &&
                                     ((uintptr_t)g.ln_res & 15) == 0 &&
                                     ((uintptr_t)g.ln_y & 15) == 0 && ((uintptr_t)g.ln_gamma & 15) == 0 &&
                                     ((uintptr_t)g.ln_beta & 15) == 0);
  return g.bt && g.M >= 1 && g.N % 64 == 0 && g.K >= kq && g.K % kq == 0 && g.lda % 8 == 0 &&
         ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.bt & 15) == 0 && !g.ce_stats && !g.dec_stats && !g.colsum &&
         ln_ok && !(g.a_ids && g.ln_gamma);
}

void gemm_breg(const GemmArgs& g, DType out, hipStream_t s) {
  require(gemm_breg_ok(g), "gemm_breg: unsupported shape or epilogue");
  if (g.ln_gamma) {
    if (out == DType::BF16) launch_ln<bf16>(g, s);
    else launch_ln<float>(g, s);
    return;
  }
  const bool wide = breg_wide(g);
  if (out == DType::BF16) {
    if (wide) launch<bf16, 64, 64, 4, 2, 2>(g, s);
    else launch<bf16, 16, 64, 8, 2, 4>(g, s);
  } else {
    if (wide) launch<float, 64, 64, 4, 2, 2>(g, s);
    else launch<float, 16, 64, 8, 2, 4>(g, s);
  }
}

void gemm_tile_b(const bf16* B, int64_t ldb, int tb, int N, int K, bf16* Bt, hipStream_t s) {
  require(N % 16 == 0 && K % 32 == 0 && ldb % 8 == 0, "gemm_tile_b: N % 16, K % 32, ldb % 8");
  if (hz::active()) {
    using namespace hz;
    op(s, "gemm_tile_b", {tb ? blk(B, K, (int64_t)N * 2, ldb * 2, RD) : blk(B, N, (int64_t)K * 2, ldb * 2, RD),
                          wr(Bt, (int64_t)N * K * 2)});
  }
  const int64_t thr = (int64_t)(N / 16) * (K / 32) * 64;
  tile_b_kernel<<<(unsigned)((thr + 255) / 256), 256, 0, s>>>(B, ldb, tb, N, K, Bt);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
