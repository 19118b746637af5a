// capgen — bf16 MFMA attention building blocks (helpers + the forward of one (batch, head)) as
// device code shared by the attention launches (attention_mfma.hip) and the fused Q/K/V projection +
// attention kernel (qkv_attn.hip).  Design notes: attention_mfma.hip header.
#pragma once
#include "attention.h"

namespace capgen {
namespace amf {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

constexpr int DK = 64;        // head size handled here
constexpr int IMG = 64 * 128;  // one [64][64] bf16 image, bytes

// image [row][64 cols]: 16-B chunk c of row k sits at chunk c ^ (((k >> 1) & 3) << 1)
__device__ __forceinline__ int swz(int k, int chunk) { return chunk ^ (((k >> 1) & 3) << 1); }

// fragment for "row" cb + (lane&15) (a COLUMN of the image) and K = image rows, permuted order
__device__ __forceinline__ bf16x8 frag_t(const char* img, int cb, int ks, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int k = ks * 32 + 4 * g + q;
  const int ch = (cb >> 3) + (p >> 1), sub = (p & 1) * 8;
  const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + k * 128 + swz(k, ch) * 16 + sub));
  const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + (k + 16) * 128 + swz(k + 16, ch) * 16 + sub));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Stage NI head slices ([L_i rows][64] bf16 from global, rows >= L_i zero) into LDS images, all
// 256 threads: every global load is issued before the first LDS write (one round trip).
template <int NI>
__device__ __forceinline__ void stage_images(char* const (&img)[NI], const bf16* const (&src)[NI],
                                             const int64_t (&ld)[NI], const int (&L)[NI], int tid) {
  uint4 v[NI][2];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u, row = c >> 3, ch = c & 7;
      v[i][u] = row < L[i] ? *reinterpret_cast<const uint4*>(src[i] + (int64_t)row * ld[i] + ch * 8)
                           : uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * u, row = c >> 3, ch = c & 7;
      *reinterpret_cast<uint4*>(img[i] + row * 128 + swz(row, ch) * 16) = v[i][u];
    }
}

// per-key validity (key-pad masks; causal is applied per row later) -> LDS bytes
__device__ __forceinline__ void stage_key_ok(unsigned char* kok, const AttnGeom& g, int b, int tid) {
  if (tid < 64) {
    const int j = tid;
    bool ok = j < g.Lk;
    if (ok && g.key_valid) ok = g.key_valid[(int64_t)(g.kv_bmod ? b % g.kv_bmod : b) * g.kv_bs + j] != 0;
    if (ok && g.key_ids) ok = g.key_ids[(int64_t)b * g.kid_bs + j] != g.pad_idx;
    kok[j] = ok;
  }
}

// 4 consecutive columns (col % 4 == 0) of one image row from f32 registers
__device__ __forceinline__ void put4(char* img, int row, int col, f32x4 v) {
  const bf16x4 b = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  *reinterpret_cast<bf16x4*>(img + row * 128 + swz(row, col >> 3) * 16 + (col & 7) * 2) = b;
}

// row fragment of an image (standard K order: 8 consecutive columns at 32ks + 8g)
__device__ __forceinline__ bf16x8 frag_r(const char* img, int row, int ks, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + row * 128 + swz(row, ks * 4 + (lane >> 4)) * 16);
}

// X[q][key] = A_row(q) . B_row(key) for this wave's 16 rows of image A (rows q0..q0+15) against
// the 64 rows of image B: s[j][r] = X[q0 + (lane&15)][16j + 4(lane>>4) + r]
__device__ __forceinline__ void scores(const char* Aimg, int q0, const char* Bimg, int lane, f32x4 (&s)[4]) {
  const bf16x8 a0 = frag_r(Aimg, q0 + (lane & 15), 0, lane), a1 = frag_r(Aimg, q0 + (lane & 15), 1, lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    s[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_r(Bimg, 16 * j + (lane & 15), 0, lane), a0, s[j], 0, 0, 0);
    s[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_r(Bimg, 16 * j + (lane & 15), 1, lane), a1, s[j], 0, 0, 0);
  }
}

// masked softmax of the 64-key rows held as in scores(); p = probabilities (pre-dropout)
__device__ __forceinline__ void softmax_rows(const AttnGeom& g, const unsigned char* kok, int q, int lane,
                                             const f32x4 (&s)[4], f32x4 (&p)[4]) {
  const float inv_t = 1.f / g.temperature;
  float mx = -INFINITY;
  f32x4 x[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = 16 * j + 4 * (lane >> 4) + r;
      const bool m = !kok[key] || (g.causal && key > g.q_pos0 + q);
      x[j][r] = m ? -INFINITY : s[j][r] * inv_t;
      mx = fmaxf(mx, x[j][r]);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      x[j][r] = expf(x[j][r] - mx);
      sum += x[j][r];
    }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) p[j][r] = x[j][r] / sum;
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& lo, const f32x4& hi) {
  return bf16x8{(bf16)lo[0], (bf16)lo[1], (bf16)lo[2], (bf16)lo[3], (bf16)hi[0], (bf16)hi[1], (bf16)hi[2], (bf16)hi[3]};
}

__device__ __forceinline__ void store4(bf16* p, f32x4 v, float mul) {
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)(v[0] * mul), (bf16)(v[1] * mul), (bf16)(v[2] * mul), (bf16)(v[3] * mul)};
}


// forward of one (batch b, head h) once Q / K / V sit in their LDS images and the key flags in kok
// (zero rows beyond Lq / Lk; the Q image needs only this wave's 16 rows): S = Q K^T -> mask ->
// softmax -> [probs] -> dropout -> O = P V.  Wave w takes query rows 16w .. 16w+15.
__device__ __forceinline__ void attn_fwd_images(const AttnGeom& g, bf16* __restrict__ o, float* __restrict__ probs,
                                                int b, int h, const char* Qimg, const char* Kimg, const char* Vimg,
                                                const unsigned char* kok) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q0 = 16 * w, q = q0 + (lane & 15);
  if (q0 >= g.Lq) return;
  f32x4 s[4], p[4];
  scores(Qimg, q0, Kimg, lane, s);
  softmax_rows(g, kok, q, lane, s, p);
  const int64_t row_idx = (((int64_t)b * g.H + h) * g.Lq + q) * g.Lk;
  if (probs && q < g.Lq) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * j + 4 * (lane >> 4) + r;
        if (key < g.Lk) probs[row_idx + key] = p[j][r];
      }
  }
  if (g.drop.seed_ptr) {
    const uint64_t seed = *g.drop.seed_ptr;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * j + 4 * (lane >> 4) + r;
        const bool keep = drop_keep(seed, g.drop.site, (uint32_t)(row_idx + key), g.drop.thresh);
        p[j][r] = keep ? p[j][r] * g.drop.scale : 0.f;
      }
  }
  // O^T[d][q] = V^T[d][key] . P^T[key][q]
  const bf16x8 pf0 = pack8(p[0], p[1]), pf1 = pack8(p[2], p[3]);
  bf16* ob = o + (int64_t)b * g.o_bs + h * DK;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t(Vimg, 16 * t, 0, lane), pf0, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t(Vimg, 16 * t, 1, lane), pf1, acc, 0, 0, 0);
    if (q < g.Lq) store4(ob + (int64_t)q * g.o_ld + 16 * t + 4 * (lane >> 4), acc, 1.f);
  }
}

// the same with the images at sm[0..3) and the key flags after them
__device__ __forceinline__ void attn_fwd_staged(const AttnGeom& g, bf16* __restrict__ o, float* __restrict__ probs,
                                                int b, int h, const char* sm) {
  attn_fwd_images(g, o, probs, b, h, sm, sm + IMG, sm + 2 * IMG, reinterpret_cast<const unsigned char*>(sm + 3 * IMG));
}

// forward of one (batch b, head h): 256 threads, sm = 3 [64][64] bf16 images + 64 key flags
__device__ __forceinline__ void attn_fwd_one(const AttnGeom& g, bf16* __restrict__ o, float* __restrict__ probs, int b,
                                             int h, char* sm) {
  char* Qimg = sm;
  char* Kimg = sm + IMG;
  char* Vimg = sm + 2 * IMG;
  unsigned char* kok = reinterpret_cast<unsigned char*>(sm + 3 * IMG);
  const int tid = threadIdx.x;
  const int bk = g.kv_bmod ? b % g.kv_bmod : b;
  {
    char* const img[3] = {Qimg, Kimg, Vimg};
    const bf16* const src[3] = {reinterpret_cast<const bf16*>(g.q) + (int64_t)b * g.q_bs + h * DK,
                                reinterpret_cast<const bf16*>(g.k) + (int64_t)bk * g.k_bs + h * DK,
                                reinterpret_cast<const bf16*>(g.v) + (int64_t)bk * g.v_bs + h * DK};
    const int64_t ld[3] = {g.q_ld, g.k_ld, g.v_ld};
    const int L[3] = {g.Lq, g.Lk, g.Lk};
    stage_images<3>(img, src, ld, L, tid);
    stage_key_ok(kok, g, b, tid);
  }
  __syncthreads();
  attn_fwd_staged(g, o, probs, b, h, sm);
}

// backward of one (batch b, head h) once K / dO / Q / V sit in their LDS images and the key flags in
// kok (zero rows beyond Lq / Lk); Pdimg / dSimg are scratch images.  256 threads; the workgroup
// barrier inside is reached by every wave.
__device__ __forceinline__ void attn_bwd_staged(const AttnGeom& g, bf16* __restrict__ dq, bf16* __restrict__ dkp,
                                                bf16* __restrict__ dvp, int b, int h, const char* Kimg,
                                                const char* dOimg, const char* Qimg, const char* Vimg, char* Pdimg,
                                                char* dSimg, const unsigned char* kok) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t qoff = (int64_t)b * g.q_bs + h * DK, koff = (int64_t)b * g.k_bs + h * DK,
                voff = (int64_t)b * g.v_bs + h * DK;
  // ---- phase 1: wave w = query rows 16w..16w+15 ----
  const int q0 = 16 * w, q = q0 + (lane & 15);
  const float inv_t = 1.f / g.temperature;
  f32x4 ds[4], pd[4];
  if (q0 < g.Lq) {
    f32x4 s[4], p[4], dp[4];
    scores(Qimg, q0, Kimg, lane, s);
    softmax_rows(g, kok, q, lane, s, p);
    scores(dOimg, q0, Vimg, lane, dp);  // d(p_dropped) = dO . V^T
    const int64_t row_idx = (((int64_t)b * g.H + h) * g.Lq + q) * g.Lk;
    const uint64_t seed = g.drop.seed_ptr ? *g.drop.seed_ptr : 0;
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = 16 * j + 4 * (lane >> 4) + r;
        float d = dp[j][r], pp = p[j][r];
        if (g.drop.seed_ptr) {
          const bool keep = drop_keep(seed, g.drop.site, (uint32_t)(row_idx + key), g.drop.thresh);
          d = keep ? d * g.drop.scale : 0.f;
          pp = keep ? pp * g.drop.scale : 0.f;
        }
        dp[j][r] = d;
        pd[j][r] = pp;
        rs += p[j][r] * d;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    const bool live = q < g.Lq;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ds[j][r] = live ? p[j][r] * (dp[j][r] - rs) : 0.f;  // softmax backward
        pd[j][r] = live ? pd[j][r] : 0.f;
      }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) ds[j] = pd[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    put4(Pdimg, q, 16 * j + 4 * (lane >> 4), pd[j]);
    put4(dSimg, q, 16 * j + 4 * (lane >> 4), ds[j]);
  }
  __syncthreads();
  if (q0 < g.Lq) {  // dQ^T[d][q] = K^T[d][key] . dS^T[key][q]
    const bf16x8 f0 = pack8(ds[0], ds[1]), f1 = pack8(ds[2], ds[3]);
    bf16* dqb = dq + qoff;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t(Kimg, 16 * t, 0, lane), f0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t(Kimg, 16 * t, 1, lane), f1, acc, 0, 0, 0);
      if (q < g.Lq) store4(dqb + (int64_t)q * g.q_ld + 16 * t + 4 * (lane >> 4), acc, inv_t);
    }
  }
  // ---- phase 2: wave w = key rows 16w..16w+15; K dimension = query rows ----
  const int k0 = 16 * w;
  if (k0 >= g.Lk) return;
  const int key = k0 + (lane & 15);
  const int nks = (g.Lq + 31) / 32;
  bf16* dvb = dvp + voff;
  bf16* dkb = dkp + koff;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x4 av = f32x4{0.f, 0.f, 0.f, 0.f}, ak = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < nks; ++ks) {
      // dV^T[d][key] = dO^T[d][q] . Pd[q][key];  dK^T[d][key] = Q^T[d][q] . dS[q][key]
      av = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t(dOimg, 16 * t, ks, lane), frag_t(Pdimg, k0, ks, lane), av,
                                                   0, 0, 0);
      ak = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_t(Qimg, 16 * t, ks, lane), frag_t(dSimg, k0, ks, lane), ak,
                                                   0, 0, 0);
    }
    if (key < g.Lk) {
      store4(dvb + (int64_t)key * g.v_ld + 16 * t + 4 * (lane >> 4), av, 1.f);
      store4(dkb + (int64_t)key * g.k_ld + 16 * t + 4 * (lane >> 4), ak, inv_t);
    }
  }
}

constexpr int kFwdSmem = 3 * IMG + 64;

}  // namespace amf
}  // namespace capgen
