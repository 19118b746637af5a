// capgen — the self-attention front of a transformer block in ONE launch (bf16): the Q/K/V
// projection of one image's rows for one head (modules.py:67-76, q_linear / k_linear / v_linear,
// no bias) followed by that head's masked attention (modules.py:16-27, attn_mfma_dev.h).
//
// One workgroup of four wave64s per (image b, head h), grid B x H.  It replaces a QKV GEMM launch
// (2304 x 1536 x 512 at C2), the dependent kernel boundary and the attention launch that re-read
// Q / K / V from memory: the projection output goes straight into the attention's LDS images (and
// to the qkv buffer the backward reads).
//
//   * the image's L <= 64 rows of X are staged in LDS once (every 16-B load issued before the first
//     LDS write), rows padded to 16 with zeros, 16-B chunks XOR-swizzled by row (conflict-free A
//     fragments);
//   * wave w computes 48 of the head's 192 projection columns (q | k | v, 64 each) for all rows:
//     its B fragments (the weight rows) are private to it, so they come straight from global
//     memory into registers, four 32-deep k-steps per batch, double buffered (the weights are
//     re-read by every image: L2 / Infinity-Cache hits).  The weights are read in a TILED copy
//     (qkv_tile_weights, kept current by the engine beside the bf16 shadow): each fragment load is
//     one coalesced 1-KB piece -- from the row-major matrix a load touched 16 rows x 64 B and the
//     launch was bound by those requests (19.3 vs 13.5 us per encoder launch, same work);
//   * v_mfma_f32_16x16x32_bf16 with swapped operands (lane = one row, 4 consecutive columns), the
//     same k order for A and B (standard order: lane group g holds k = 8g .. 8g+7);
//   * the f32 results are rounded to bf16 once -- exactly the values a bf16 GEMM store would leave
//     in the qkv buffer -- and written to the buffer and to the three [64][64] LDS images;
//   * then attn_fwd_staged (attention_mfma.hip's forward body) runs on the images.
#include <cstdlib>

#include "qkv_attn.h"

#include "attn_mfma_dev.h"
#include "hazard.h"

namespace capgen {
using namespace amf;

namespace {

constexpr int QD = 512;       // model width handled here (K of the projection)
constexpr int QKS = QD / 32;  // 32-deep k-steps
constexpr int QKB = 4;        // k-steps per register batch of weight fragments

__device__ __forceinline__ int xswz(int row, int chunk) { return chunk ^ (row & 15); }
__device__ int32_t g_qa_dummy[64];  // target of the absent key-mask inputs (never used as a value)

// The image's rows of a [L][512] bf16 operand (X in the front, dA in the backward) into the LDS
// staging area by LDS-DMA (round 6): one buffer_load_dwordx4 ... lds per 1-KB row, lane l's 16 B
// landing at slot l of the row -- slot l holds chunk l ^ (row & 15), the XOR swizzle applied through
// the source offset.  Rows >= L get an offset past the buffer's num_records (zeros land), so every
// staged row up to 16 LT is written.  Nothing passes through VGPRs: the register staging it replaces
// held the image's rows in 4 LT uint4 per lane (48 VGPRs at LT = 3) across the weight loads.  The
// issuing wave's s_waitcnt vmcnt(0) + a workgroup barrier make the rows visible (the caller).
// `s_nop 4`: the VALU-written M0 / voff before an LDS-DMA need wait states hipcc does not pad into an
// asm statement (gemm_tile.h Op::dma).
template <int LT>
__device__ __forceinline__ void dma_rows(const bf16* rows, int64_t ld, int L, char* xs, int w, int lane) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(rows), 0, (int)((int64_t)L * ld * 2), 0x00020000);
#pragma unroll
  for (int j = 0; j < 4 * LT; ++j) {
    const int row = w + 4 * j;
    const uint32_t voff = row < L ? (uint32_t)(((int64_t)row * ld + (lane ^ (row & 15)) * 8) * 2) : 0x80000000u;
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rs), "s"(0u),
                 "{m0}"((unsigned)(uintptr_t)(xs + row * (QD * 2)))
                 : "memory");
  }
}

__device__ __forceinline__ void bf8_to_f(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = __uint_as_float(w[e] << 16);
    f[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}

// NP = 3: self attention, q | k | v all projected from X (L = Lq = Lk rows);
// NP = 1: cross attention, only q projected (Lq rows of X), K / V staged from g.k / g.v (Lk rows)
template <int LT, int NP>  // LT: query-row tiles of 16 (Lq <= 16 LT)
__global__ void __launch_bounds__(256) qkv_attn_kernel(QkvAttn a) {
  __shared__ __attribute__((aligned(16))) char sm[kFwdSmem];
  __shared__ __attribute__((aligned(16))) char xs[LT * 16 * QD * 2];
  StampScope stamp_scope(a.g.stamp);
  if (a.g.prio) __builtin_amdgcn_s_setprio(3);
  const AttnGeom& g = a.g;
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NF = NP;  // 16-column fragments per wave (48 or 16 of the 64 NP columns)
  const int L = g.Lq;     // rows of X (query rows)
  const bf16* xb = a.X + (int64_t)b * L * a.ldx;

  // ---- first weight batch, X rows (rows past L not loaded: in the step that beat re-reading the last
  // row, round 4),
  // key flags; then the LDS writes: X (rows >= L zero), zeroed attention images.
  // Projection: wave w -> columns 48w .. 48w+47 of [q_h | k_h | v_h]. ----
  const int fr = lane & 15, fg = lane >> 4;
  // (tiled weights: fragment f of this wave = 16-row block j of W, one 1-KB piece per k-step)
  const bf16* wrow[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int c = 16 * NF * w + 16 * f, which = c >> 6, within = c & 63;
    wrow[f] = a.W + ((int64_t)((which * QD + h * DK + within) >> 4) * QKS * 64 + lane) * 8;
  }
  bf16x8 bq[2][QKB][NF];
#pragma unroll
  for (int kk = 0; kk < QKB; ++kk)
#pragma unroll
    for (int f = 0; f < NF; ++f) bq[0][kk][f] = *reinterpret_cast<const bf16x8*>(wrow[f] + 512 * kk);
  {
    dma_rows<LT>(xb, a.ldx, L, xs, w, lane);  // X rows -> LDS, nothing through registers
    // cross attention: K / V head slices from memory (rows < Lk)
    uint4 kv[2][2];
    if constexpr (NP == 1) {
      const int bk = g.kv_bmod ? b % g.kv_bmod : b;
      const bf16* src[2] = {reinterpret_cast<const bf16*>(g.k) + (int64_t)bk * g.k_bs + h * DK,
                            reinterpret_cast<const bf16*>(g.v) + (int64_t)bk * g.v_bs + h * DK};
      const int64_t ld[2] = {g.k_ld, g.v_ld};
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = tid + 256 * u, row = c >> 3, ch = c & 7;
          kv[i][u] = row < g.Lk
                         ? *reinterpret_cast<const uint4*>(src[i] + (int64_t)min(row, g.Lk - 1) * ld[i] + ch * 8)
                         : uint4{0u, 0u, 0u, 0u};
        }
    }
    // key flags (stage_key_ok's two dependent conditional loads, as one unconditional batch)
    int kid = 0, kvl = 1;
    if (w == 0) {
      const int j = min(lane, g.Lk - 1);
      const int bk = g.kv_bmod ? b % g.kv_bmod : b;
      kid = opaque(g.key_ids ? g.key_ids : g_qa_dummy)[g.key_ids ? (int64_t)b * g.kid_bs + j : lane];
      kvl = opaque(g.key_valid ? g.key_valid : reinterpret_cast<const uint8_t*>(g_qa_dummy))[
          g.key_valid ? (int64_t)bk * g.kv_bs + j : lane];
    }
#pragma unroll
    for (int u = 0; u < NP * IMG / 16 / 256; ++u)
      reinterpret_cast<uint4*>(sm)[tid + 256 * u] = uint4{0u, 0u, 0u, 0u};
    if constexpr (NP == 1) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = tid + 256 * u, row = c >> 3, ch = c & 7;
          *reinterpret_cast<uint4*>(sm + (1 + i) * IMG + row * 128 + swz(row, ch) * 16) =
              row < g.Lk ? kv[i][u] : uint4{0u, 0u, 0u, 0u};
        }
    }
    if (w == 0)
      reinterpret_cast<unsigned char*>(sm + 3 * IMG)[lane] =
          lane < g.Lk && (!g.key_valid || kvl != 0) && (!g.key_ids || kid != g.pad_idx);
  }
  f32x4 acc[LT][NF];
#pragma unroll
  for (int i = 0; i < LT; ++i)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's X rows have landed (and its weights)
  __syncthreads();  // X staged
#pragma unroll
  for (int grp = 0; grp < QKS / QKB; ++grp) {
    const int cur = grp & 1;
    if (grp + 1 < QKS / QKB) {
#pragma unroll
      for (int kk = 0; kk < QKB; ++kk)
#pragma unroll
        for (int f = 0; f < NF; ++f)
          bq[cur ^ 1][kk][f] = *reinterpret_cast<const bf16x8*>(wrow[f] + 512 * ((grp + 1) * QKB + kk));
    }
    // the next batch's loads all issue before this batch's MFMAs (hipcc otherwise interleaves them
    // with partial waits and keeps only ~5 of the 12 in flight)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < QKB; ++kk) {
      const int ks = grp * QKB + kk;
#pragma unroll
      for (int i = 0; i < LT; ++i) {
        const int row = 16 * i + fr;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + row * (QD * 2) + xswz(row, 4 * ks + fg) * 16);
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][kk][f], af, acc[i][f], 0, 0, 0);
      }
    }
  }

  // ---- bf16 results -> the qkv buffer (backward) and the LDS images (attention) ----
  // lane holds C[row 16i + fr][col 16 NF w + 16f + 4fg + 0..3]
  bf16* qkvb = a.qkv ? a.qkv + (int64_t)b * L * a.ldqkv : nullptr;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int c = 16 * NF * w + 16 * f + 4 * fg, which = c >> 6, within = c & 63;
    char* img = sm + which * IMG;
#pragma unroll
    for (int i = 0; i < LT; ++i) {
      const int row = 16 * i + fr;
      const f32x4 v = acc[i][f];
      const bf16x4 r4 = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      if (row < L) {
        if (a.qkv) *reinterpret_cast<bf16x4*>(qkvb + (int64_t)row * a.ldqkv + which * QD + h * DK + within) = r4;
        *reinterpret_cast<bf16x4*>(img + row * 128 + swz(row, within >> 3) * 16 + (within & 7) * 2) = r4;
      }
    }
  }
  __syncthreads();
  attn_fwd_staged(g, a.o, nullptr, b, h, sm);
}

// ---- the output side of the attention backward (QkvBwd) ----
// Phase 0 as the cross front's projection (qkv_attn_kernel<LT, 1>): the image's dA rows staged in LDS,
// wave w computes dO columns 16w .. 16w+15 of head h over every row with its 16 tiled Wo^T fragments
// loaded in one batch; the bf16-rounded dO (the value a bf16 GEMM would store) goes to the dO image.
// The K / Q / V rows are loaded into registers with the weights and written into their images only
// after the projection, over the dA staging area (LDS: max(dA rows, 5 images) + the dO image).
template <int LT>
__global__ void __launch_bounds__(256) qkv_attn_bwd_kernel(QkvBwd a) {
  constexpr int XS = LT * 16 * QD * 2;
  constexpr int RA = XS > 5 * IMG ? XS : 5 * IMG;
  __shared__ __attribute__((aligned(16))) char sm[RA + IMG + 64];
  char* xs = sm;
  char* Kimg = sm;
  char* Qimg = sm + IMG;
  char* Vimg = sm + 2 * IMG;
  char* Pdimg = sm + 3 * IMG;
  char* dSimg = sm + 4 * IMG;
  char* dOimg = sm + RA;
  unsigned char* kok = reinterpret_cast<unsigned char*>(sm + RA + IMG);
  const AttnGeom& g = a.g;
  StampScope stamp_scope(g.stamp);
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int L = g.Lq;
  // every global load first: weights (16 tiled fragments), dA rows, K / Q / V rows, key flags
  const bf16* wrow = a.Wt + ((int64_t)((h * DK + 16 * w) >> 4) * QKS * 64 + lane) * 8;
  bf16x8 bq[QKS];
#pragma unroll
  for (int ks = 0; ks < QKS; ++ks) bq[ks] = *reinterpret_cast<const bf16x8*>(wrow + 512 * ks);
  dma_rows<LT>(a.dA + (int64_t)b * L * a.ldda, a.ldda, L, xs, w, lane);  // dA rows -> LDS (no registers)
  const int bk = g.kv_bmod ? b % g.kv_bmod : b;
  const bf16* src[3] = {reinterpret_cast<const bf16*>(g.k) + (int64_t)bk * g.k_bs + h * DK,
                        reinterpret_cast<const bf16*>(g.q) + (int64_t)b * g.q_bs + h * DK,
                        reinterpret_cast<const bf16*>(g.v) + (int64_t)bk * g.v_bs + h * DK};
  const int64_t ld[3] = {g.k_ld, g.q_ld, g.v_ld};
  const int Ls[3] = {g.Lk, g.Lq, g.Lk};
  uint4 kqv[3][2];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u, row = c >> 3, ch = c & 7;
      kqv[i][u] = row < Ls[i]
                      ? *reinterpret_cast<const uint4*>(src[i] + (int64_t)min(row, Ls[i] - 1) * ld[i] + ch * 8)
                      : uint4{0u, 0u, 0u, 0u};
    }
  int kid = 0, kvl = 1;
  if (w == 0) {
    const int j = min(lane, g.Lk - 1);
    kid = opaque(g.key_ids ? g.key_ids : g_qa_dummy)[g.key_ids ? (int64_t)b * g.kid_bs + j : lane];
    kvl = opaque(g.key_valid ? g.key_valid : reinterpret_cast<const uint8_t*>(g_qa_dummy))[
        g.key_valid ? (int64_t)bk * g.kv_bs + j : lane];
  }
  // the dO image zeroed (rows >= 16 LT are never projected); the dA rows (rows >= L zero) landing by DMA
#pragma unroll
  for (int u = 0; u < 2; ++u) reinterpret_cast<uint4*>(dOimg)[tid + 256 * u] = uint4{0u, 0u, 0u, 0u};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's dA rows have landed (and its loads)
  __syncthreads();
  f32x4 acc[LT];
#pragma unroll
  for (int i = 0; i < LT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < QKS; ++ks)
#pragma unroll
    for (int i = 0; i < LT; ++i) {
      const int row = 16 * i + fr;
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + row * (QD * 2) + xswz(row, 4 * ks + fg) * 16);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ks], af, acc[i], 0, 0, 0);
    }
  // lane holds dO[row 16i + fr][col 16w + 4fg + 0..3] (rows >= L: zero, from the zero dA rows)
#pragma unroll
  for (int i = 0; i < LT; ++i) {
    const int row = 16 * i + fr, col = 16 * w + 4 * fg;
    const bf16x4 r4 = {(bf16)acc[i][0], (bf16)acc[i][1], (bf16)acc[i][2], (bf16)acc[i][3]};
    *reinterpret_cast<bf16x4*>(dOimg + row * 128 + swz(row, col >> 3) * 16 + (col & 7) * 2) = r4;
  }
  __syncthreads();  // (the dA staging area is free: K / Q / V images over it)
  {
    char* const img[3] = {Kimg, Qimg, Vimg};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = tid + 256 * u, row = c >> 3, ch = c & 7;
        *reinterpret_cast<uint4*>(img[i] + row * 128 + swz(row, ch) * 16) = row < Ls[i] ? kqv[i][u] : uint4{0u, 0u, 0u, 0u};
      }
    if (w == 0) kok[lane] = lane < g.Lk && (!g.key_valid || kvl != 0) && (!g.key_ids || kid != g.pad_idx);
  }
  __syncthreads();
  attn_bwd_staged(g, a.dq, a.dk, a.dv, b, h, Kimg, dOimg, Qimg, Vimg, Pdimg, dSimg, kok);
}

// W^T tiled: a workgroup transposes a 32 (k) x 64 (n) block of src through LDS -- coalesced 16-B row
// loads in, 16-B piece stores out (the per-lane gather of 8 strided bf16 it replaces took 4.8 us per
// 512 x 512 matrix in the step)
__global__ void __launch_bounds__(256) tile_weights_t_kernel(const bf16* __restrict__ src, int64_t ld,
                                                             bf16* __restrict__ dst) {
  __shared__ bf16 t[32][64 + 8];
  const int tid = threadIdx.x, k0 = blockIdx.y * 32, n0 = blockIdx.x * 64;
  {
    const int row = tid >> 3, ch = tid & 7;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + (int64_t)(k0 + row) * ld + n0 + ch * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) t[row][ch * 8 + e] = v[e];
  }
  __syncthreads();
  const int jj = tid >> 6, lane = tid & 63;
  const int nl = 16 * jj + (lane & 15), kk = 8 * (lane >> 4);
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = t[kk + e][nl];  // dst row n = column n of src
  const int64_t piece = (int64_t)(n0 / 16 + jj) * QKS + k0 / 32;
  reinterpret_cast<bf16x8*>(dst)[piece * 64 + lane] = o;
}
__global__ void tile_weights_kernel(const bf16* __restrict__ src, int64_t n, int64_t ld, bf16* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // 16-B piece of dst
  if (i >= n) return;
  const int lane = (int)(i & 63), ks = (int)((i >> 6) % QKS);
  const int64_t j = (i >> 6) / QKS;
  const uint4 v = *reinterpret_cast<const uint4*>(src + (16 * j + (lane & 15)) * ld + 32 * ks + 8 * (lane >> 4));
  reinterpret_cast<uint4*>(dst)[i] = v;
}

}  // namespace

void qkv_tile_weights(const bf16* src, int R, int64_t ld, bf16* dst, hipStream_t s) {
  require(R > 0 && R % 16 == 0 && ld % 8 == 0 && ld >= QD, "qkv_tile_weights: R % 16 == 0, ld >= 512");
  if (hz::active()) {
    using namespace hz;
    hz::op(s, "qkv_tile_weights", {blk(src, R, QD * 2, ld * 2, RD), wr(dst, (int64_t)R * QD * 2)});
  }
  const int64_t n = (int64_t)R * QD / 8;
  tile_weights_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(src, n, ld, dst);
  CAPGEN_HIP(hipGetLastError());
}

bool qkv_attn_ok(const QkvAttn& a) {
  const AttnGeom& g = a.g;
  const bool shape = a.cross ? (g.Lk >= 1 && g.Lk <= 64 && g.k_ld % 8 == 0 && g.v_ld % 8 == 0 && g.k_bs % 8 == 0 &&
                                g.v_bs % 8 == 0)
                             : (g.Lq == g.Lk && g.kv_bmod == 0);
  return shape && g.dk == DK && g.H * DK == QD && a.d == QD && g.Lq >= 1 && g.Lq <= 64 && !g.kv_row && a.W &&
         a.ldx % 8 == 0 && a.ldqkv % 8 == 0 && g.o_ld % 8 == 0 && g.o_bs % 8 == 0;
}

void qkv_attn_fwd(const QkvAttn& a_in, hipStream_t s) {
  QkvAttn a = a_in;
  require(qkv_attn_ok(a), "qkv_attn_fwd: unsupported geometry (head size 64, d = 512, self attention, L <= 64)");
  const AttnGeom& g = a.g;
  if (hz::active()) {
    using namespace hz;
    const int L = g.Lq;
    const int np = a.cross ? 1 : 3, Bk = g.kv_bmod > 0 ? std::min(g.B, g.kv_bmod) : g.B;
    const Rgn r[] = {rows_blk(a.X, g.B, L, (int64_t)L * a.ldx, a.ldx, a.d, 2, RD),
                     rd(a.W, (int64_t)np * QD * QD * 2),
                     blk(g.key_valid, Bk, g.Lk, g.kv_bs, RD), blk(g.key_ids, g.B, (int64_t)g.Lk * 4, g.kid_bs * 4, RD),
                     rows_blk(a.cross ? g.k : nullptr, Bk, g.Lk, g.k_bs, g.k_ld, a.d, 2, RD),
                     rows_blk(a.cross ? g.v : nullptr, Bk, g.Lk, g.v_bs, g.v_ld, a.d, 2, RD),
                     rd(g.drop.seed_ptr, 8), rows_blk(a.qkv, g.B, L, (int64_t)L * a.ldqkv, a.ldqkv, np * a.d, 2, WR),
                     rows_blk(a.o, g.B, L, g.o_bs, g.o_ld, a.d, 2, WR)};
    op(s, "qkv_attn", r, sizeof r / sizeof r[0]);
  }
  const int lt = (a.g.Lq + 15) / 16;
  const dim3 grid(a.g.B * a.g.H);
  if (a.cross) {
    switch (lt) {
      case 1: qkv_attn_kernel<1, 1><<<grid, 256, 0, s>>>(a); break;
      case 2: qkv_attn_kernel<2, 1><<<grid, 256, 0, s>>>(a); break;
      case 3: qkv_attn_kernel<3, 1><<<grid, 256, 0, s>>>(a); break;
      default: qkv_attn_kernel<4, 1><<<grid, 256, 0, s>>>(a); break;
    }
  } else {
    switch (lt) {
      case 1: qkv_attn_kernel<1, 3><<<grid, 256, 0, s>>>(a); break;
      case 2: qkv_attn_kernel<2, 3><<<grid, 256, 0, s>>>(a); break;
      case 3: qkv_attn_kernel<3, 3><<<grid, 256, 0, s>>>(a); break;
      default: qkv_attn_kernel<4, 3><<<grid, 256, 0, s>>>(a); break;
    }
  }
  CAPGEN_HIP(hipGetLastError());
}

bool qkv_bwd_ok(const QkvBwd& a) {
  const AttnGeom& g = a.g;
  // (kv_bmod: K / V shared by several images -- decode only; the staged backward writes dk / dv per image)
  return g.dk == DK && g.H * DK == QD && g.Lq >= 1 && g.Lq <= 64 && g.Lk >= 1 && g.Lk <= 64 && !g.kv_row &&
         g.kv_bmod == 0 && a.Wt &&
         a.dA && a.dq && a.dk && a.dv && a.ldda % 8 == 0 && g.q_ld % 8 == 0 && g.k_ld % 8 == 0 && g.v_ld % 8 == 0 &&
         g.q_bs % 8 == 0 && g.k_bs % 8 == 0 && g.v_bs % 8 == 0;
}

void qkv_attn_bwd(const QkvBwd& a_in, hipStream_t s) {
  QkvBwd a = a_in;
  require(qkv_bwd_ok(a), "qkv_attn_bwd: unsupported geometry (head size 64, d = 512, Lq / Lk <= 64)");
  const AttnGeom& g = a.g;
  if (hz::active()) {
    using namespace hz;
    const int Bk = g.kv_bmod > 0 ? std::min(g.B, g.kv_bmod) : g.B;
    const int64_t w = (int64_t)g.H * g.dk;
    const Rgn r[] = {rows_blk(a.dA, g.B, g.Lq, (int64_t)g.Lq * a.ldda, a.ldda, QD, 2, RD),
                     rd(a.Wt, (int64_t)QD * QD * 2),
                     rows_blk(g.q, g.B, g.Lq, g.q_bs, g.q_ld, w, 2, RD), rows_blk(g.k, Bk, g.Lk, g.k_bs, g.k_ld, w, 2, RD),
                     rows_blk(g.v, Bk, g.Lk, g.v_bs, g.v_ld, w, 2, RD), blk(g.key_valid, Bk, g.Lk, g.kv_bs, RD),
                     blk(g.key_ids, g.B, (int64_t)g.Lk * 4, g.kid_bs * 4, RD), rd(g.drop.seed_ptr, 8),
                     rows_blk(a.dq, g.B, g.Lq, g.q_bs, g.q_ld, w, 2, WR),
                     rows_blk(a.dk, Bk, g.Lk, g.k_bs, g.k_ld, w, 2, WR),
                     rows_blk(a.dv, Bk, g.Lk, g.v_bs, g.v_ld, w, 2, WR)};
    op(s, "qkv_attn_bwd", r, sizeof r / sizeof r[0]);
  }
  const dim3 grid(g.B * g.H);
  switch ((g.Lq + 15) / 16) {
    case 1: qkv_attn_bwd_kernel<1><<<grid, 256, 0, s>>>(a); break;
    case 2: qkv_attn_bwd_kernel<2><<<grid, 256, 0, s>>>(a); break;
    case 3: qkv_attn_bwd_kernel<3><<<grid, 256, 0, s>>>(a); break;
    default: qkv_attn_bwd_kernel<4><<<grid, 256, 0, s>>>(a); break;
  }
  CAPGEN_HIP(hipGetLastError());
}

void qkv_tile_weights_t(const bf16* src, int64_t ld, bf16* dst, hipStream_t s) {
  require(ld % 8 == 0 && ld >= QD, "qkv_tile_weights_t: ld >= 512");
  if (hz::active()) {
    using namespace hz;
    hz::op(s, "qkv_tile_weights_t", {blk(src, QD, QD * 2, ld * 2, RD), wr(dst, (int64_t)QD * QD * 2)});
  }
  tile_weights_t_kernel<<<dim3(QD / 64, QD / 32), 256, 0, s>>>(src, ld, dst);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
