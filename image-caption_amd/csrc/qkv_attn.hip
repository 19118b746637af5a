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
//     re-read by every image: L2 / Infinity-Cache hits);
//   * v_mfma_f32_16x16x32_bf16 with swapped operands (lane = one row, 4 consecutive columns), the
//     same k order for A and B (standard order: lane group g holds k = 8g .. 8g+7);
//   * the f32 results are rounded to bf16 once -- exactly the values a bf16 GEMM store would leave
//     in the qkv buffer -- and written to the buffer and to the three [64][64] LDS images;
//   * then attn_fwd_staged (attention_mfma.hip's forward body) runs on the images.
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
  const bf16* xb = a.X + (int64_t)b * (a.x_bs >= 0 ? a.x_bs : (int64_t)L * a.ldx);

  // ---- first weight batch, X rows (clamped row, unconditional: no load waits at a branch join),
  // key flags; then the LDS writes: X (rows >= L zero), zeroed attention images.
  // Projection: wave w -> columns 48w .. 48w+47 of [q_h | k_h | v_h]. ----
  const int fr = lane & 15, fg = lane >> 4;
  const bf16* wrow[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int c = 16 * NF * w + 16 * f + fr, which = c >> 6, within = c & 63;
    wrow[f] = a.W + (int64_t)(which * QD + h * DK + within) * a.ldw + 8 * fg;
  }
  bf16x8 bq[2][QKB][NF];
#pragma unroll
  for (int kk = 0; kk < QKB; ++kk)
#pragma unroll
    for (int f = 0; f < NF; ++f) bq[0][kk][f] = *reinterpret_cast<const bf16x8*>(wrow[f] + 32 * kk);
  {
    constexpr int CH = LT * 16 * QD / 8;  // 16-B chunks of the staged rows
    constexpr int PER = CH / 256;
    uint4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + 256 * u, row = c / (QD / 8), ch = c % (QD / 8);
      v[u] = *reinterpret_cast<const uint4*>(xb + (int64_t)min(row, L - 1) * a.ldx + ch * 8);
    }
    // cross attention: K / V head slices from memory (rows < Lk, clamped, unconditional)
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
          kv[i][u] = *reinterpret_cast<const uint4*>(src[i] + (int64_t)min(row, g.Lk - 1) * ld[i] + ch * 8);
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
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + 256 * u, row = c / (QD / 8), ch = c % (QD / 8);
      *reinterpret_cast<uint4*>(xs + row * (QD * 2) + xswz(row, ch) * 16) = row < L ? v[u] : uint4{0u, 0u, 0u, 0u};
    }
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
  __syncthreads();  // X staged
#pragma unroll
  for (int grp = 0; grp < QKS / QKB; ++grp) {
    const int cur = grp & 1;
    if (grp + 1 < QKS / QKB) {
#pragma unroll
      for (int kk = 0; kk < QKB; ++kk)
#pragma unroll
        for (int f = 0; f < NF; ++f)
          bq[cur ^ 1][kk][f] = *reinterpret_cast<const bf16x8*>(wrow[f] + 32 * ((grp + 1) * QKB + kk));
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

// ---- KV-cached decode step, self attention (QkvDecode) ----
// Phase 1 as qkv_attn_kernel<1, 3> (rows r = j * B + image, j < kb <= 16): the image's rows of x in
// LDS, wave w projects 48 of the head's 192 columns.  The bf16 q / k / v go to LDS; k / v also to
// every row's cache slot at position t.  Phase 2 as attn_decode_bf16_kernel's single mode (lane =
// (key slot jr = lane / 8, 16-B chunk c = lane % 8), the 8-chunk dot, softmax and P.V reduced across
// lanes with the same DPP / shuffle order): wave w runs rows j = w, w + 4, ...; key p < t from cache
// row kv_row[r][p], key t from the LDS copy of the fresh k / v.
template <int NIT>  // key slots of 8: t + 1 <= 8 NIT
__global__ void __launch_bounds__(256) qkv_decode_kernel(QkvDecode a) {
  __shared__ __attribute__((aligned(16))) char xs[16 * QD * 2];
  __shared__ __attribute__((aligned(16))) bf16 qkv_s[3][16][DK];
  StampScope stamp_scope(a.stamp);
  if (a.prio) __builtin_amdgcn_s_setprio(3);
  const int img = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kb = a.kb, t = a.t;
  const int64_t rstride = (int64_t)a.B * QD;  // x / o row of beam j: + j * B * d
  const bf16* xb = a.X + (int64_t)img * QD;
  const int fr = lane & 15, fg = lane >> 4;
  const bf16* wrow[3];
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const int c = 48 * w + 16 * f + fr, which = c >> 6, within = c & 63;
    wrow[f] = a.W + (int64_t)(which * QD + h * DK + within) * QD + 8 * fg;
  }
  bf16x8 bq[2][QKB][3];
#pragma unroll
  for (int kk = 0; kk < QKB; ++kk)
#pragma unroll
    for (int f = 0; f < 3; ++f) bq[0][kk][f] = *reinterpret_cast<const bf16x8*>(wrow[f] + 32 * kk);
  {
    constexpr int PER = 16 * QD / 8 / 256;
    uint4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + 256 * u, row = c / (QD / 8), ch = c % (QD / 8);
      v[u] = *reinterpret_cast<const uint4*>(xb + (int64_t)min(row, kb - 1) * rstride + ch * 8);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + 256 * u, row = c / (QD / 8), ch = c % (QD / 8);
      *reinterpret_cast<uint4*>(xs + row * (QD * 2) + xswz(row, ch) * 16) = row < kb ? v[u] : uint4{0u, 0u, 0u, 0u};
    }
  }
  f32x4 acc[3];
#pragma unroll
  for (int f = 0; f < 3; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
#pragma unroll
  for (int grp = 0; grp < QKS / QKB; ++grp) {
    const int cur = grp & 1;
    if (grp + 1 < QKS / QKB) {
#pragma unroll
      for (int kk = 0; kk < QKB; ++kk)
#pragma unroll
        for (int f = 0; f < 3; ++f)
          bq[cur ^ 1][kk][f] = *reinterpret_cast<const bf16x8*>(wrow[f] + 32 * ((grp + 1) * QKB + kk));
    }
    __builtin_amdgcn_sched_barrier(0);  // (as in qkv_attn_kernel)
#pragma unroll
    for (int kk = 0; kk < QKB; ++kk) {
      const int ks = grp * QKB + kk;
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + fr * (QD * 2) + xswz(fr, 4 * ks + fg) * 16);
#pragma unroll
      for (int f = 0; f < 3; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][kk][f], af, acc[f], 0, 0, 0);
    }
  }
  // lane holds [row fr][col 48w + 16f + 4fg + 0..3]: bf16 -> LDS (q, k, v) and k / v -> the cache
#pragma unroll
  for (int f = 0; f < 3; ++f) {
    const int c = 48 * w + 16 * f + 4 * fg, which = c >> 6, within = c & 63;
    const f32x4 v = acc[f];
    const bf16x4 r4 = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    if (fr < kb) {
      *reinterpret_cast<bf16x4*>(&qkv_s[which][fr][within]) = r4;
      if (which > 0) {
        const int64_t r = (int64_t)fr * a.B + img;
        *reinterpret_cast<bf16x4*>(a.cache + r * a.c_ld + (int64_t)t * 2 * QD + (which - 1) * QD + h * DK + within) = r4;
      }
    }
  }
  __syncthreads();
  // ---- phase 2: one row per wave at a time ----
  const int jr = lane >> 3, c = lane & 7;
  const float inv_t = 1.f / a.temperature;
  for (int j = w; j < kb; j += 4) {
    const int64_t r = (int64_t)j * a.B + img;
    // key slot p = jr + 8 it: its cache row (the beam it descends from), loaded up front
    uint4 kr[NIT], vr[NIT];
    bool kin[NIT];
    int idp[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int p = jr + 8 * it;
      kin[it] = p <= t;
      const int pc = min(p, t);
      const int64_t src = a.kv_row ? a.kv_row[r * a.kv_row_ld + pc] : r;
      const bf16* kp = a.cache + src * a.c_ld + (int64_t)pc * 2 * QD + h * DK + c * 8;
      kr[it] = *reinterpret_cast<const uint4*>(kp);
      vr[it] = *reinterpret_cast<const uint4*>(kp + QD);
      idp[it] = a.ids[r * a.ids_ld + pc];
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it)
      if (jr + 8 * it == t) {  // position t: this row's fresh k / v (LDS, not the just-written cache)
        kr[it] = *reinterpret_cast<const uint4*>(&qkv_s[1][j][c * 8]);
        vr[it] = *reinterpret_cast<const uint4*>(&qkv_s[2][j][c * 8]);
      }
    float q[8];
    bf8_to_f(*reinterpret_cast<const uint4*>(&qkv_s[0][j][c * 8]), q);
    float sc[NIT];
    float mx = -INFINITY;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      float k[8];
      bf8_to_f(kr[it], k);
      float dot = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) dot = fmaf(q[e] * inv_t, k[e], dot);
      dot += dpp_f<kDppXor1>(dot);
      dot += dpp_f<kDppXor2>(dot);
      dot += dpp_f<kDppHalfMirror>(dot);
      sc[it] = kin[it] && idp[it] != a.pad_idx ? dot : -INFINITY;
      mx = fmaxf(mx, sc[it]);
    }
    mx = fmaxf(mx, dpp_f<kDppRor8>(mx));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      sc[it] = kin[it] ? expf(sc[it] - mx) : 0.f;
      sum += sc[it];
    }
    sum += dpp_f<kDppRor8>(sum);
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
    float ov[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const float pr = sc[it] * inv;
      float v[8];
      bf8_to_f(vr[it], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) ov[e] = fmaf(pr, v[e], ov[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ov[e] += dpp_f<kDppRor8>(ov[e]);
      ov[e] += __shfl_xor(ov[e], 16, 64);
      ov[e] += __shfl_xor(ov[e], 32, 64);
    }
    if (jr == 0) {
      const bf16x8 ob = {(bf16)ov[0], (bf16)ov[1], (bf16)ov[2], (bf16)ov[3], (bf16)ov[4], (bf16)ov[5], (bf16)ov[6], (bf16)ov[7]};
      *reinterpret_cast<bf16x8*>(a.o + r * QD + h * DK + c * 8) = ob;
    }
  }
}

}  // namespace

bool qkv_attn_ok(const QkvAttn& a) {
  const AttnGeom& g = a.g;
  const bool shape = a.cross ? (g.Lk >= 1 && g.Lk <= 64 && g.k_ld % 8 == 0 && g.v_ld % 8 == 0 && g.k_bs % 8 == 0 &&
                                g.v_bs % 8 == 0)
                             : (g.Lq == g.Lk && g.kv_bmod == 0);
  return shape && g.dk == DK && g.H * DK == QD && a.d == QD && g.Lq >= 1 && g.Lq <= 64 && !g.kv_row &&
         a.ldx % 8 == 0 && a.ldw % 8 == 0 && a.ldqkv % 8 == 0 && g.o_ld % 8 == 0 && g.o_bs % 8 == 0;
}

void qkv_attn_fwd(const QkvAttn& a, hipStream_t s) {
  require(qkv_attn_ok(a), "qkv_attn_fwd: unsupported geometry (head size 64, d = 512, self attention, L <= 64)");
  const AttnGeom& g = a.g;
  if (hz::active()) {
    using namespace hz;
    const int L = g.Lq;
    const int np = a.cross ? 1 : 3, Bk = g.kv_bmod > 0 ? std::min(g.B, g.kv_bmod) : g.B;
    const Rgn r[] = {rows_blk(a.X, g.B, L, a.x_bs >= 0 ? a.x_bs : (int64_t)L * a.ldx, a.ldx, a.d, 2, RD),
                     rd(a.W, (int64_t)np * a.d * a.ldw * 2),
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

}  // namespace capgen

namespace capgen {

bool qkv_decode_ok(const QkvDecode& a) {
  return a.d == QD && a.H * DK == QD && a.kb >= 1 && a.kb <= 16 && a.t >= 0 && a.t < 64 && a.ids && a.c_ld % 8 == 0;
}

void qkv_decode_self(const QkvDecode& a, hipStream_t s) {
  require(qkv_decode_ok(a), "qkv_decode_self: unsupported geometry (d = 512, head size 64, <= 16 rows per image, t < 64)");
  if (hz::active()) {
    using namespace hz;
    const int64_t R = (int64_t)a.B * a.kb;
    const Rgn r[] = {rd(a.X, R * a.d * 2), rd(a.W, (int64_t)3 * a.d * a.d * 2), rd(a.kv_row, R * a.kv_row_ld * 4),
                     rd(a.ids, R * a.ids_ld * 4), blk(a.cache, R, (int64_t)(a.t + 1) * 2 * a.d * 2, a.c_ld * 2, ACC),
                     wr(a.o, R * a.d * 2)};
    op(s, "qkv_decode_self", r, sizeof r / sizeof r[0]);
  }
  const dim3 grid(a.B * a.H);
  const int n = a.t + 1;
  if (n <= 24) qkv_decode_kernel<3><<<grid, 256, 0, s>>>(a);
  else if (n <= 40) qkv_decode_kernel<5><<<grid, 256, 0, s>>>(a);
  else qkv_decode_kernel<8><<<grid, 256, 0, s>>>(a);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
