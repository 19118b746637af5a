// capgen — fused masked attention for short sequences (Lq, Lk <= 64), one workgroup per
// (batch, head).  Whole Q/K/V head tiles are staged in LDS as f32 (a 36x64 tile is 9 KB);
// scores, softmax, dropout and P.V never touch HBM.  The softmax of one query row is one
// wave64 (lane = key) reduced with cross-lane shuffles.  HBM traffic: the Q/K/V reads, the O
// write and (for backward / attention_list) the f32 probabilities.
//
// Products are VALU f32 FMAs over 16-B LDS reads: score tiles are 2x2 register blocks
// (4 ds_read_b128 per 16 FMAs), P.V / dS.K / P^T.dO produce 4 consecutive head columns per
// thread (one broadcast scalar + one ds_read_b128 per 4 FMAs).  Rows are padded to dk+4
// floats (16-B aligned, 4-bank skew), the row count to even so 2x2 blocks need no branch.
// Every dot product runs in natural index order, so results match a sequential f32 sum.
//
// Semantics (modules.py:16-27, 67-92): s = (q / temperature) . k^T; masked_fill(-inf);
// softmax; dropout; o = p . v.  Backward recomputes the dropout mask from the counter RNG.
#include <cstdlib>
#include <algorithm>

#include <type_traits>

#include "attention.h"
#include "hazard.h"

namespace capgen {

constexpr int AT_THREADS = 256;

__device__ __forceinline__ bool key_masked(const AttnGeom& g, int b, int i, int j) {
  if (g.causal && j > g.q_pos0 + i) return true;
  if (g.key_valid && !g.key_valid[(int64_t)(g.kv_bmod ? b % g.kv_bmod : b) * g.kv_bs + j]) return true;
  if (g.key_ids && g.key_ids[(int64_t)b * g.kid_bs + j] == g.pad_idx) return true;
  return false;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float dot4(float4 a, float4 b, float acc) {
  acc = fmaf(a.x, b.x, acc);
  acc = fmaf(a.y, b.y, acc);
  acc = fmaf(a.z, b.z, acc);
  return fmaf(a.w, b.w, acc);
}
__device__ __forceinline__ void axpy4(float s, float4 v, float4& acc) {
  acc.x = fmaf(s, v.x, acc.x);
  acc.y = fmaf(s, v.y, acc.y);
  acc.z = fmaf(s, v.z, acc.z);
  acc.w = fmaf(s, v.w, acc.w);
}
template <typename T>
__device__ __forceinline__ void st4(T* p, float4 v, float mul) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = float4{v.x * mul, v.y * mul, v.z * mul, v.w * mul};
  } else {
    typedef __attribute__((ext_vector_type(4))) __bf16 b4;
    *reinterpret_cast<b4*>(p) = b4{(bf16)(v.x * mul), (bf16)(v.y * mul), (bf16)(v.z * mul), (bf16)(v.w * mul)};
  }
}

// rows x dk tile -> LDS [rows_padded][ldd] f32 (x / div), zero pad row when rows is odd
template <typename T>
__device__ __forceinline__ void stage_rows(float* dst, int ldd, const T* src, int64_t ld, int rows, int dk,
                                           float div, int tid, const int32_t* rowmap = nullptr, int64_t row_bs = 0,
                                           int base_row = 0) {
  constexpr int V = 16 / sizeof(T);
  const int cpr = dk / V;
  for (int c = tid; c < rows * cpr; c += AT_THREADS) {
    const int r = c / cpr, d = (c % cpr) * V;
    float x[V];
    // rowmap (AttnGeom::kv_row): row r of this batch is stored in batch rowmap[r]
    const int64_t roff = rowmap ? (int64_t)(rowmap[r] - base_row) * row_bs : 0;
    load_f<T, V>(src + roff + (int64_t)r * ld + d, x);
#pragma unroll
    for (int e = 0; e < V; ++e) dst[r * ldd + d + e] = div == 1.f ? x[e] : x[e] / div;
  }
  if (rows & 1)
    for (int d = tid; d < dk; d += AT_THREADS) dst[rows * ldd + d] = 0.f;
}

// C[i][j] = sum_d X[i][d] Y[j][d] for i < R, j < Cn (2x2 register blocks)
__device__ __forceinline__ void gram(const float* X, const float* Y, int ldd, int R, int Cn, int dk, float* C,
                                     int ldc, int tid) {
  const int ti = (R + 1) >> 1, tj = (Cn + 1) >> 1;
  for (int c = tid; c < ti * tj; c += AT_THREADS) {
    const int i0 = (c / tj) * 2, j0 = (c % tj) * 2;
    const float* x0 = X + i0 * ldd;
    const float* y0 = Y + j0 * ldd;
    float a00 = 0.f, a01 = 0.f, a10 = 0.f, a11 = 0.f;
    for (int d = 0; d < dk; d += 4) {
      const float4 p0 = ld4(x0 + d), p1 = ld4(x0 + ldd + d);
      const float4 q0 = ld4(y0 + d), q1 = ld4(y0 + ldd + d);
      a00 = dot4(p0, q0, a00);
      a01 = dot4(p0, q1, a01);
      a10 = dot4(p1, q0, a10);
      a11 = dot4(p1, q1, a11);
    }
    C[i0 * ldc + j0] = a00;
    if (j0 + 1 < Cn) C[i0 * ldc + j0 + 1] = a01;
    if (i0 + 1 < R) {
      C[(i0 + 1) * ldc + j0] = a10;
      if (j0 + 1 < Cn) C[(i0 + 1) * ldc + j0 + 1] = a11;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(AT_THREADS) attn_fwd_kernel(AttnGeom g, T* __restrict__ o,
                                                              float* __restrict__ probs) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H;
  const int Lq = g.Lq, Lk = g.Lk, dk = g.dk, ldd = dk + 4, lds_s = Lk + 1;
  const int Lq2 = (Lq + 1) & ~1, Lk2 = (Lk + 1) & ~1;
  float* Qs = sm;
  float* Ks = Qs + Lq2 * ldd;
  float* Vs = Ks + Lk2 * ldd;
  float* S = Vs + Lk2 * ldd;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  const T* q = reinterpret_cast<const T*>(g.q) + (int64_t)b * g.q_bs + h * dk;
  const int bk = g.kv_bmod ? b % g.kv_bmod : b;
  const T* k = reinterpret_cast<const T*>(g.k) + (int64_t)bk * g.k_bs + h * dk;
  const T* v = reinterpret_cast<const T*>(g.v) + (int64_t)bk * g.v_bs + h * dk;
  stage_rows<T>(Qs, ldd, q, g.q_ld, Lq, dk, g.temperature, tid);
  const int32_t* rowmap = g.kv_row ? g.kv_row + (int64_t)b * g.kv_row_ld : nullptr;
  stage_rows<T>(Ks, ldd, k, g.k_ld, Lk, dk, 1.f, tid, rowmap, g.k_bs, bk);
  stage_rows<T>(Vs, ldd, v, g.v_ld, Lk, dk, 1.f, tid, rowmap, g.v_bs, bk);
  __syncthreads();

  gram(Qs, Ks, ldd, Lq, Lk, dk, S, lds_s, tid);
  __syncthreads();

  const uint64_t seed = g.drop.seed_ptr ? *g.drop.seed_ptr : 0;
  for (int i = wave; i < Lq; i += AT_THREADS / 64) {
    const int j = lane;
    float s = -INFINITY;
    if (j < Lk) s = key_masked(g, b, i, j) ? -INFINITY : S[i * lds_s + j];
    const float mx = wave_max(s);
    const float e = j < Lk ? expf(s - mx) : 0.f;
    const float sum = wave_sum(e);
    if (j < Lk) {
      float p = e / sum;
      const int64_t idx = (((int64_t)b * g.H + h) * Lq + i) * Lk + j;
      if (probs) probs[idx] = p;
      if (g.drop.seed_ptr) p = drop_keep(seed, g.drop.site, (uint32_t)idx, g.drop.thresh) ? p * g.drop.scale : 0.f;
      S[i * lds_s + j] = p;
    }
  }
  __syncthreads();

  T* ob = o + (int64_t)b * g.o_bs + h * dk;
  const int d4n = dk >> 2;
  for (int c = tid; c < Lq * d4n; c += AT_THREADS) {
    const int i = c / d4n, d = (c % d4n) * 4;
    const float* pi = S + i * lds_s;
    float4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < Lk; ++j) axpy4(pi[j], ld4(Vs + j * ldd + d), acc);
    st4<T>(ob + (int64_t)i * g.o_ld + d, acc, 1.f);
  }
}

template <typename T>
__global__ void __launch_bounds__(AT_THREADS) attn_bwd_kernel(AttnGeom g, const float* __restrict__ probs,
                                                              const T* __restrict__ dout, T* __restrict__ dq,
                                                              T* __restrict__ dkp, T* __restrict__ dvp) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H;
  const int Lq = g.Lq, Lk = g.Lk, dk = g.dk, ldd = dk + 4, lds_s = Lk + 1;
  const int Lq2 = (Lq + 1) & ~1, Lk2 = (Lk + 1) & ~1;
  float* Qs = sm;                 // q / temperature
  float* Ks = Qs + Lq2 * ldd;
  float* Vs = Ks + Lk2 * ldd;
  float* dO = Vs + Lk2 * ldd;
  float* Ps = dO + Lq2 * ldd;     // p, then dropped p
  float* Ds = Ps + Lq * lds_s;    // d(p_dropped), then d(score)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  const int64_t qoff = (int64_t)b * g.q_bs + h * dk, koff = (int64_t)b * g.k_bs + h * dk,
                voff = (int64_t)b * g.v_bs + h * dk, ooff = (int64_t)b * g.o_bs + h * dk;
  stage_rows<T>(Qs, ldd, reinterpret_cast<const T*>(g.q) + qoff, g.q_ld, Lq, dk, g.temperature, tid);
  stage_rows<T>(Ks, ldd, reinterpret_cast<const T*>(g.k) + koff, g.k_ld, Lk, dk, 1.f, tid);
  stage_rows<T>(Vs, ldd, reinterpret_cast<const T*>(g.v) + voff, g.v_ld, Lk, dk, 1.f, tid);
  stage_rows<T>(dO, ldd, dout + ooff, g.o_ld, Lq, dk, 1.f, tid);
  const float* pb = probs + ((int64_t)b * g.H + h) * Lq * Lk;
  for (int c = tid; c < Lq * Lk; c += AT_THREADS) Ps[(c / Lk) * lds_s + c % Lk] = pb[c];
  __syncthreads();

  gram(dO, Vs, ldd, Lq, Lk, dk, Ds, lds_s, tid);  // d(p_dropped) = dO . V^T
  __syncthreads();

  const uint64_t seed = g.drop.seed_ptr ? *g.drop.seed_ptr : 0;
  for (int i = wave; i < Lq; i += AT_THREADS / 64) {
    const int j = lane;
    float p = 0.f, dp = 0.f, pd = 0.f;
    if (j < Lk) {
      p = Ps[i * lds_s + j];
      dp = Ds[i * lds_s + j];
      pd = p;
      if (g.drop.seed_ptr) {
        const int64_t idx = (((int64_t)b * g.H + h) * Lq + i) * Lk + j;
        const bool keep = drop_keep(seed, g.drop.site, (uint32_t)idx, g.drop.thresh);
        dp = keep ? dp * g.drop.scale : 0.f;
        pd = keep ? p * g.drop.scale : 0.f;
      }
    }
    const float rs = wave_sum(p * dp);
    if (j < Lk) {
      Ds[i * lds_s + j] = p * (dp - rs);  // softmax backward
      Ps[i * lds_s + j] = pd;
    }
  }
  __syncthreads();

  const int d4n = dk >> 2;
  T* dkb = dkp + koff;
  T* dvb = dvp + voff;
  for (int c = tid; c < Lk * d4n; c += AT_THREADS) {
    const int j = c / d4n, d = (c % d4n) * 4;
    float4 av = {0.f, 0.f, 0.f, 0.f}, ak = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < Lq; ++i) {
      axpy4(Ps[i * lds_s + j], ld4(dO + i * ldd + d), av);
      axpy4(Ds[i * lds_s + j], ld4(Qs + i * ldd + d), ak);
    }
    st4<T>(dvb + (int64_t)j * g.v_ld + d, av, 1.f);
    st4<T>(dkb + (int64_t)j * g.k_ld + d, ak, 1.f);
  }
  T* dqb = dq + qoff;
  for (int c = tid; c < Lq * d4n; c += AT_THREADS) {
    const int i = c / d4n, d = (c % d4n) * 4;
    const float* di = Ds + i * lds_s;
    float4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < Lk; ++j) axpy4(di[j], ld4(Ks + j * ldd + d), acc);
    // (dS . K) / temperature, as the division backward of q / temperature
    float4 r = {acc.x / g.temperature, acc.y / g.temperature, acc.z / g.temperature, acc.w / g.temperature};
    st4<T>(dqb + (int64_t)i * g.q_ld + d, r, 1.f);
  }
}

static bool group_decode_on();
// Single-query attention (KV-cached decode step, model.py:101-200 with a cache): one wave64 per
// (row, head).  Every global load is issued up front -- the row-table entry of key `lane`, then
// that key's K row (lane = key, 16-B loads) and every V row (lane = head dim, one coalesced row per
// instruction, its base taken from the table by readlane) -- so a wave pays two memory round trips
// (round 1 staged V through LDS behind a barrier and loaded K after it: four).  Arithmetic as
// attn_fwd_kernel's, in the same order (q / temperature first; d-sequential dots; the same wave
// butterflies; j-sequential P.V), so f32 results are bit-identical to it.  No dropout (decode).
template <typename T, int LKM>
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnGeom g, T* __restrict__ o, float* __restrict__ probs) {
  __shared__ float qsh[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int w = blockIdx.x * 4 + wv;
  if (w >= g.B * g.H) return;  // no workgroup barrier below
  const int b = w / g.H, h = w % g.H;
  const int bk = g.kv_bmod ? b % g.kv_bmod : b;
  const T* kb = reinterpret_cast<const T*>(g.k) + (int64_t)bk * g.k_bs + h * 64;
  const T* vb = reinterpret_cast<const T*>(g.v) + (int64_t)bk * g.v_bs + h * 64;
  constexpr int V = 16 / sizeof(T);
  typedef typename Vec16<T>::type VT;
  const int Lk = g.Lk, j = lane;
  const int rj = g.kv_row && j < Lk ? g.kv_row[(int64_t)b * g.kv_row_ld + j] - bk : 0;
  const bool live = j < Lk && !key_masked(g, b, 0, j);
  const float qv = to_f(reinterpret_cast<const T*>(g.q)[(int64_t)b * g.q_bs + h * 64 + lane]) / g.temperature;
  VT kr[64 / V];
  if (live) {
    const T* kp = kb + (int64_t)rj * g.k_bs + (int64_t)j * g.k_ld;
#pragma unroll
    for (int c = 0; c < 64 / V; ++c) kr[c] = *reinterpret_cast<const VT*>(kp + c * V);
  }
  T vr[LKM];
#pragma unroll
  for (int jj = 0; jj < LKM; ++jj)
    if (jj < Lk) {
      const int r = g.kv_row ? __builtin_amdgcn_readlane(rj, jj) : 0;
      vr[jj] = vb[(int64_t)r * g.v_bs + (int64_t)jj * g.v_ld + lane];
    }
  qsh[wv][lane] = qv;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float s = -INFINITY;
  if (live) {
    const T* kx = reinterpret_cast<const T*>(kr);
    float acc = 0.f;
#pragma unroll
    for (int d = 0; d < 64; ++d) acc = fmaf(qsh[wv][d], to_f(kx[d]), acc);
    s = acc;
  }
  const float mx = wave_max(s);
  const float e = j < Lk ? expf(s - mx) : 0.f;
  const float sum = wave_sum(e);
  const float p = e / sum;
  if (probs && j < Lk) probs[(((int64_t)b * g.H + h)) * Lk + j] = p;
  float acc = 0.f;
#pragma unroll
  for (int jj = 0; jj < LKM; ++jj)
    if (jj < Lk) acc = fmaf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), jj)), to_f(vr[jj]), acc);
  o[(int64_t)b * g.o_bs + h * 64 + lane] = from_f<T>(acc);
}

// Cross-attention decode step when several rows read one image's K/V (beam search: rows
// j*kv_bmod + i all attend over image i; no kv_row indirection, no causal / key-id mask): one
// wave per (image, head) loads the image's K (lane = key) and V (lane = head dim) and the queries
// of its G = B / kv_bmod rows once, up front, then runs the queries one after another.  Each
// query's arithmetic is attn_decode_kernel's, in the same order (bit-identical results); the
// image's K/V leave L2 once per (image, head), not G times.
template <typename T, int LKM, int GM>
__global__ void __launch_bounds__(256) attn_decode_group_kernel(AttnGeom g, int G, T* __restrict__ o,
                                                                float* __restrict__ probs) {
  __shared__ float qsh[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nimg = g.kv_bmod, w = blockIdx.x * 4 + wv;
  if (w >= nimg * g.H) return;  // no workgroup barrier below
  const int i = w / g.H, h = w % g.H;
  const T* kb = reinterpret_cast<const T*>(g.k) + (int64_t)i * g.k_bs + h * 64;
  const T* vb = reinterpret_cast<const T*>(g.v) + (int64_t)i * g.v_bs + h * 64;
  constexpr int V = 16 / sizeof(T);
  typedef typename Vec16<T>::type VT;
  const int Lk = g.Lk, j = lane;
  const bool live = j < Lk && !key_masked(g, i, 0, j);  // key mask of image i (b % kv_bmod = i)
  VT kr[64 / V];
  if (j < Lk) {
#pragma unroll
    for (int c = 0; c < 64 / V; ++c) kr[c] = *reinterpret_cast<const VT*>(kb + (int64_t)j * g.k_ld + c * V);
  }
  T vr[LKM];
#pragma unroll
  for (int jj = 0; jj < LKM; ++jj)
    if (jj < Lk) vr[jj] = vb[(int64_t)jj * g.v_ld + lane];
  float qr[GM];
#pragma unroll
  for (int qi = 0; qi < GM; ++qi)
    if (qi < G)
      qr[qi] = to_f(reinterpret_cast<const T*>(g.q)[(int64_t)(qi * nimg + i) * g.q_bs + h * 64 + lane]) / g.temperature;
  const T* kx = reinterpret_cast<const T*>(kr);
#pragma unroll
  for (int qi = 0; qi < GM; ++qi) {
    if (qi >= G) continue;  // (a constant trip count: the loop unrolls and qr stays in registers)
    const int b = qi * nimg + i;
    qsh[wv][lane] = qr[qi];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float s = -INFINITY;
    if (live) {
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < 64; ++d) acc = fmaf(qsh[wv][d], to_f(kx[d]), acc);
      s = acc;
    }
    const float mx = wave_max(s);
    const float e = j < Lk ? expf(s - mx) : 0.f;
    const float sum = wave_sum(e);
    const float p = e / sum;
    if (probs && j < Lk) probs[(((int64_t)b * g.H + h)) * Lk + j] = p;
    float acc = 0.f;
#pragma unroll
    for (int jj = 0; jj < LKM; ++jj)
      if (jj < Lk) acc = fmaf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), jj)), to_f(vr[jj]), acc);
    o[(int64_t)b * g.o_bs + h * 64 + lane] = from_f<T>(acc);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // this query's qsh reads before the next write
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// bf16 KV-cached decode step, coalesced: lane = (key slot jr = lane / 8, 16-B chunk c = lane % 8),
// so one load instruction brings 8 whole 128-B K (or V) rows of a head (lane = key, as in the f32
// kernel above, touches 64 rows per instruction and is bound by the address unit).  Keys j = jr,
// jr + 8, ... ; the 8-chunk dot, the softmax and the P.V sums reduce across lanes.  Single mode
// (G = 1): wave = (query row, head), K/V rows through the beam row table.  Group mode (G > 1, beam
// cross attention): workgroup = (image, head), wave wv runs queries wv, wv + 4, ... of the image's
// G rows (K/V of the image: L1/L2 hits after the first wave).  Sums in a different order than the
// f32 kernel (bf16 operands; the f32 path keeps the order pinned to attn_fwd_kernel).
__device__ __forceinline__ void bf16x8_to_f(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = __uint_as_float(w[e] << 16);
    f[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}
// Group mode with kv_lds (CAPGEN_DECODE_GROUP_LDS, default on): the workgroup stages the image's K/V
// rows of the head in LDS once (one coalesced pass over Lk x 128 B each) and every wave takes its
// chunks from there -- without it each of the workgroup's waves loads the same rows from L1/L2
// (4 waves x 2048 (image, head) workgroups at C4).  Same per-lane values, same sums: bit-identical.
template <int NIT>
__global__ void __launch_bounds__(512) attn_decode_bf16_kernel(AttnGeom g, int G, bf16* __restrict__ o,
                                                               float* __restrict__ probs, int kv_lds) {
  __shared__ uint4 kvs[2][64 * 8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, jr = lane >> 3, c = lane & 7;
  const bool group = G > 1;
  int b0, h, bk, qfirst, qstep;
  if (group) {  // workgroup = (image, head); queries qi*nimg + image, qi = wv, wv + waves, ...
    const int i = blockIdx.x / g.H;
    h = blockIdx.x % g.H, bk = i, b0 = i, qfirst = wv, qstep = blockDim.x >> 6;
  } else {
    const int w = blockIdx.x * 4 + wv;
    if (w >= g.B * g.H) return;  // no workgroup barrier in this kernel
    b0 = w / g.H, h = w % g.H, bk = g.kv_bmod ? b0 % g.kv_bmod : b0, qfirst = 0, qstep = 1;
  }
  const int Lk = g.Lk;
  const bf16* kb = reinterpret_cast<const bf16*>(g.k) + (int64_t)bk * g.k_bs + h * 64 + c * 8;
  const bf16* vb = reinterpret_cast<const bf16*>(g.v) + (int64_t)bk * g.v_bs + h * 64 + c * 8;
  // the query chunk of query qi (clamped to a valid query: the prefetch past the last one is unused)
  auto qload = [&](int qi) {
    const int b = group ? min(qi, G - 1) * g.kv_bmod + b0 : b0;
    return *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(g.q) + (int64_t)b * g.q_bs + h * 64 + c * 8);
  };
  // the first query is loaded with the K/V rows, each later one while the previous query computes
  // (group mode: a wave runs up to 8 queries; a load at the top of each iteration was one more
  // memory round trip per query)
  uint4 qnext = qload(qfirst);
  // beam row table: lane l holds the cache row of key l (single mode only)
  const int rl = (!group && g.kv_row && lane < Lk) ? g.kv_row[(int64_t)b0 * g.kv_row_ld + lane] - bk : 0;
  uint4 kr[NIT], vr[NIT];
  bool kin[NIT];
  if (group && kv_lds) {  // (uniform: the whole workgroup takes this branch, so the barrier is safe)
    const bf16* k0 = kb - c * 8;
    const bf16* v0 = vb - c * 8;
    for (int idx = threadIdx.x; idx < Lk * 8; idx += blockDim.x) {
      const int j = idx >> 3, cc = idx & 7;
      kvs[0][idx] = *reinterpret_cast<const uint4*>(k0 + (int64_t)j * g.k_ld + cc * 8);
      kvs[1][idx] = *reinterpret_cast<const uint4*>(v0 + (int64_t)j * g.v_ld + cc * 8);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int j = jr + 8 * it;
      kin[it] = j < Lk;
      kr[it] = kin[it] ? kvs[0][j * 8 + c] : make_uint4(0, 0, 0, 0);
      vr[it] = kin[it] ? kvs[1][j * 8 + c] : make_uint4(0, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int j = jr + 8 * it;
      kin[it] = j < Lk;
      const int r = g.kv_row ? __shfl(rl, j < 64 ? j : 0, 64) : 0;
      if (kin[it]) {
        kr[it] = *reinterpret_cast<const uint4*>(kb + (int64_t)r * g.k_bs + (int64_t)j * g.k_ld);
        vr[it] = *reinterpret_cast<const uint4*>(vb + (int64_t)r * g.v_bs + (int64_t)j * g.v_ld);
      } else {
        kr[it] = vr[it] = make_uint4(0, 0, 0, 0);
      }
    }
  }
  const float inv_t = 1.f / g.temperature;
  for (int qi = qfirst; qi < G; qi += qstep) {
    const int b = group ? qi * g.kv_bmod + b0 : b0;
    float q[8];
    bf16x8_to_f(qnext, q);
    qnext = qload(qi + qstep);
    float s[NIT];
    float mx = -INFINITY;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      float k[8];
      bf16x8_to_f(kr[it], k);
      float acc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc = fmaf(q[e] * inv_t, k[e], acc);
      acc += dpp_f<kDppXor1>(acc);  // the 8 chunks of key j: lanes 8 jr .. 8 jr + 7
      acc += dpp_f<kDppXor2>(acc);
      acc += dpp_f<kDppHalfMirror>(acc);
      const int j = jr + 8 * it;
      s[it] = kin[it] && !key_masked(g, b, 0, j) ? acc : -INFINITY;
      mx = fmaxf(mx, s[it]);
    }
    mx = fmaxf(mx, dpp_f<kDppRor8>(mx));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      s[it] = kin[it] ? expf(s[it] - mx) : 0.f;
      sum += s[it];
    }
    sum += dpp_f<kDppRor8>(sum);
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const float p = s[it] * inv;
      if (probs && c == 0 && kin[it]) probs[((int64_t)b * g.H + h) * Lk + jr + 8 * it] = p;
      float v[8];
      bf16x8_to_f(vr[it], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(p, v[e], acc[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      acc[e] += dpp_f<kDppRor8>(acc[e]);  // lane ^ 8: the same chunk c of the next key slot
      acc[e] += __shfl_xor(acc[e], 16, 64);
      acc[e] += __shfl_xor(acc[e], 32, 64);
    }
    if (jr == 0) {
      uint4 u;
      uint32_t* w = reinterpret_cast<uint32_t*>(&u);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16 lo = (bf16)acc[2 * e], hi = (bf16)acc[2 * e + 1];
        w[e] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
      }
      *reinterpret_cast<uint4*>(o + (int64_t)b * g.o_bs + h * 64 + c * 8) = u;
    }
  }
}

template <typename T>
static void launch_decode(const AttnGeom& g, T* o, float* probs, hipStream_t s) {
  const int G = g.kv_bmod > 0 ? g.B / g.kv_bmod : 1;
  const bool grouped = G >= 2 && G <= 16 && g.B % g.kv_bmod == 0 && !g.kv_row && !g.causal && !g.key_ids &&
                       group_decode_on();
  if constexpr (std::is_same<T, bf16>::value) {
    if (((g.q_bs | g.k_bs | g.v_bs | g.k_ld | g.v_ld | g.o_bs) % 8) == 0) {
      const int blocks = grouped ? g.kv_bmod * g.H : (g.B * g.H + 3) / 4;
      const int Gk = grouped ? G : 1;
      // grouped: 2 waves share the image's queries.  C4 beam 5, two alternating rounds per setting
      // (round 3): 1 wave 14.7-15.7 ms/batch, 2 waves 14.2-14.5, 4 waves 14.6-14.7, 8 waves 15.1-15.2
      // (one wave per beam row, round 2: 25.1 vs 18.8 us/launch)
      const int nt = grouped ? 128 : 256;
      const int kv_lds = knob(Knob::DecodeGroupLds) ? 1 : 0;
      const int lds = grouped ? kv_lds : 0;
      if (g.Lk <= 24) attn_decode_bf16_kernel<3><<<blocks, nt, 0, s>>>(g, Gk, o, probs, lds);
      else if (g.Lk <= 40) attn_decode_bf16_kernel<5><<<blocks, nt, 0, s>>>(g, Gk, o, probs, lds);
      else attn_decode_bf16_kernel<8><<<blocks, nt, 0, s>>>(g, Gk, o, probs, lds);
      CAPGEN_HIP(hipGetLastError());
      return;
    }
  }
  if (grouped) {
    const int blocks = (g.kv_bmod * g.H + 3) / 4;  // one wave per (image, head): its rows' K/V read once
    auto go = [&](auto lkm, auto gm) {
      attn_decode_group_kernel<T, decltype(lkm)::value, decltype(gm)::value><<<blocks, 256, 0, s>>>(g, G, o, probs);
    };
    using I32 = std::integral_constant<int, 32>;
    using I64 = std::integral_constant<int, 64>;
    if (G <= 4) g.Lk <= 32 ? go(I32{}, std::integral_constant<int, 4>{}) : go(I64{}, std::integral_constant<int, 4>{});
    else if (G <= 8) g.Lk <= 32 ? go(I32{}, std::integral_constant<int, 8>{}) : go(I64{}, std::integral_constant<int, 8>{});
    else g.Lk <= 32 ? go(I32{}, std::integral_constant<int, 16>{}) : go(I64{}, std::integral_constant<int, 16>{});
  } else {
    const int blocks = (g.B * g.H + 3) / 4;
    if (g.Lk <= 32) attn_decode_kernel<T, 32><<<blocks, 256, 0, s>>>(g, o, probs);
    else attn_decode_kernel<T, 64><<<blocks, 256, 0, s>>>(g, o, probs);
  }
  CAPGEN_HIP(hipGetLastError());
}

__global__ void head_mean_kernel(const float* __restrict__ probs, int B, int H, int Lq, int Lk, int row,
                                 float* __restrict__ out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= B * Lk) return;
  int b = c / Lk, j = c % Lk;
  float acc = 0.f;
  for (int h = 0; h < H; ++h) acc += probs[(((int64_t)b * H + h) * Lq + row) * Lk + j];
  out[c] = acc / (float)H;
}

// grouped decode (an image's beam rows in one workgroup, its K/V read once): always on
static bool group_decode_on() { return true; }

static void check_geom(const AttnGeom& g) {
  require(g.Lq >= 1 && g.Lq <= 64 && g.Lk >= 1 && g.Lk <= 64, "attention: Lq/Lk must be in [1, 64]");
  require(g.dk % 8 == 0 && g.dk <= 128, "attention: head size must be a multiple of 8 and <= 128");
}

static size_t fwd_smem(const AttnGeom& g) {
  const size_t ldd = g.dk + 4, Lq2 = (g.Lq + 1) & ~1, Lk2 = (g.Lk + 1) & ~1;
  return sizeof(float) * (Lq2 * ldd + 2 * Lk2 * ldd + g.Lq * (g.Lk + 1));
}
static size_t bwd_smem(const AttnGeom& g) {
  const size_t ldd = g.dk + 4, Lq2 = (g.Lq + 1) & ~1, Lk2 = (g.Lk + 1) & ~1;
  return sizeof(float) * (2 * Lq2 * ldd + 2 * Lk2 * ldd + 2 * g.Lq * (g.Lk + 1));
}

template <typename K>
static void allow_big_lds(K kernel) {
  static bool done = false;  // per instantiation
  if (!done) {
    CAPGEN_HIP(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    done = true;
  }
}

// the device bytes one attention launch touches (hazard checker, hazard.h)
static void hz_attention(const AttnGeom& g, DType t, hipStream_t s, const char* name, const void* o, const float* probs,
                         const void* dout, const void* dq, const void* dk, const void* dv) {
  using namespace hz;
  const int64_t e = dsize(t), w = (int64_t)g.H * g.dk;
  const int Bk = g.kv_bmod > 0 ? std::min(g.B, g.kv_bmod) : g.B;
  const Rgn r[] = {
      rows_blk(g.q, g.B, g.Lq, g.q_bs, g.q_ld, w, e, RD), rows_blk(g.k, Bk, g.Lk, g.k_bs, g.k_ld, w, e, RD),
      rows_blk(g.v, Bk, g.Lk, g.v_bs, g.v_ld, w, e, RD), blk(g.key_valid, Bk, g.Lk, g.kv_bs, RD),
      blk(g.key_ids, Bk, (int64_t)g.Lk * 4, g.kid_bs * 4, RD), rd(g.drop.seed_ptr, 8),
      rows_blk(o, g.B, g.Lq, g.o_bs, g.o_ld, w, e, WR),
      rd(probs, dout ? (int64_t)g.B * g.H * g.Lq * g.Lk * 4 : 0),  // backward reads the saved probabilities
      wr(dout ? nullptr : probs, (int64_t)g.B * g.H * g.Lq * g.Lk * 4),
      rows_blk(dout, g.B, g.Lq, g.o_bs, g.o_ld, w, e, RD), rows_blk(dq, g.B, g.Lq, g.q_bs, g.q_ld, w, e, WR),
      rows_blk(dk, Bk, g.Lk, g.k_bs, g.k_ld, w, e, WR), rows_blk(dv, Bk, g.Lk, g.v_bs, g.v_ld, w, e, WR)};
  op(s, name, r, sizeof r / sizeof r[0]);
}

void attention_fwd(const AttnGeom& g, void* o, float* probs, DType t, hipStream_t s) {
  if (skip_mask() & 2) return;
  check_geom(g);
  if (hz::active() && !g.kv_row) hz_attention(g, t, s, "attention_fwd", o, probs, nullptr, nullptr, nullptr, nullptr);
  if (g.Lq == 1 && g.dk == 64 && g.drop.seed_ptr == nullptr && g.q_ld % 8 == 0 && g.k_ld % 8 == 0 &&
      ((g.q_bs | g.k_bs) % 8) == 0) {  // KV-cached decode step
    if (t == DType::F32) launch_decode<float>(g, (float*)o, probs, s);
    else launch_decode<bf16>(g, (bf16*)o, probs, s);
    return;
  }
  if (t == DType::BF16 && !g.kv_row && attention_mfma_ok(g)) return attention_fwd_mfma(g, (bf16*)o, probs, s);
  const size_t smem = fwd_smem(g);
  require(smem <= 160 * 1024, "attention_fwd: LDS budget exceeded");
  dim3 grid(g.B * g.H);
  if (t == DType::F32) {
    allow_big_lds(attn_fwd_kernel<float>);
    attn_fwd_kernel<float><<<grid, AT_THREADS, smem, s>>>(g, (float*)o, probs);
  } else {
    allow_big_lds(attn_fwd_kernel<bf16>);
    attn_fwd_kernel<bf16><<<grid, AT_THREADS, smem, s>>>(g, (bf16*)o, probs);
  }
  CAPGEN_HIP(hipGetLastError());
}

void attention_bwd(const AttnGeom& g, const float* probs, const void* dout, void* dq, void* dk, void* dv, DType t,
                   hipStream_t s) {
  if (skip_mask() & 8) return;
  check_geom(g);
  if (hz::active()) hz_attention(g, t, s, "attention_bwd", nullptr, probs, dout, dq, dk, dv);
  if (t == DType::BF16 && attention_mfma_ok(g))
    return attention_bwd_mfma(g, (const bf16*)dout, (bf16*)dq, (bf16*)dk, (bf16*)dv, s);
  const size_t smem = bwd_smem(g);
  require(smem <= 160 * 1024, "attention_bwd: LDS budget exceeded (head size too large)");
  dim3 grid(g.B * g.H);
  if (t == DType::F32) {
    allow_big_lds(attn_bwd_kernel<float>);
    attn_bwd_kernel<float><<<grid, AT_THREADS, smem, s>>>(g, probs, (const float*)dout, (float*)dq, (float*)dk,
                                                          (float*)dv);
  } else {
    allow_big_lds(attn_bwd_kernel<bf16>);
    attn_bwd_kernel<bf16><<<grid, AT_THREADS, smem, s>>>(g, probs, (const bf16*)dout, (bf16*)dq, (bf16*)dk,
                                                         (bf16*)dv);
  }
  CAPGEN_HIP(hipGetLastError());
}

void attention_head_mean(const float* probs, int B, int H, int Lq, int Lk, int row, float* out, hipStream_t s) {
  int n = B * Lk;
  head_mean_kernel<<<(n + 255) / 256, 256, 0, s>>>(probs, B, H, Lq, Lk, row, out);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
