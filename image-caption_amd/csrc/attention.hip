// capgen — fused masked attention for short sequences (Lq, Lk <= 64), one workgroup per
// (batch, head).  Whole Q/K/V head tiles are staged in LDS as f32 (a 36x64 tile is 9 KB),
// scores/softmax/dropout/PV never touch HBM; the softmax of one query row is one wave64
// (lane = key) reduced with cross-lane shuffles.  The only HBM traffic is the Q/K/V read,
// the O write and (for backward / attention_list) the f32 probabilities.
//
// Semantics (modules.py:16-27, 67-92): s = (q / temperature) . k^T; masked_fill(-inf);
// softmax; dropout; o = p . v.  Backward recomputes the dropout mask from the counter RNG.
#include "attention.h"

namespace capgen {

constexpr int AT_THREADS = 256;

__device__ __forceinline__ bool key_masked(const AttnGeom& g, int b, int i, int j) {
  if (g.causal && j > g.q_pos0 + i) return true;
  if (g.key_valid && !g.key_valid[(int64_t)(g.kv_bmod ? b % g.kv_bmod : b) * g.kv_bs + j]) return true;
  if (g.key_ids && g.key_ids[(int64_t)b * g.kid_bs + j] == g.pad_idx) return true;
  return false;
}

template <typename T>
__device__ __forceinline__ void stage_rows(float* dst, int ldd, const T* src, int64_t ld, int rows,
                                           int dk, float mul, int tid) {
  // rows x dk tile, 8-element (bf16) / 4-element (f32) chunks along dk
  constexpr int V = 16 / sizeof(T);
  const int cpr = dk / V;
  for (int c = tid; c < rows * cpr; c += AT_THREADS) {
    int r = c / cpr, d = (c % cpr) * V;
    float x[V];
    load_f<T, V>(src + (int64_t)r * ld + d, x);
#pragma unroll
    for (int e = 0; e < V; ++e) dst[r * ldd + d + e] = mul == 1.f ? x[e] : x[e] / mul;
  }
}

template <typename T>
__global__ void __launch_bounds__(AT_THREADS) attn_fwd_kernel(AttnGeom g, T* __restrict__ o,
                                                              float* __restrict__ probs) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H;
  const int Lq = g.Lq, Lk = g.Lk, dk = g.dk, ldd = dk + 1, lds_s = Lk + 1;
  float* Qs = sm;
  float* Ks = Qs + Lq * ldd;
  float* Vs = Ks + Lk * ldd;
  float* S = Vs + Lk * ldd;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  const T* q = reinterpret_cast<const T*>(g.q) + (int64_t)b * g.q_bs + h * dk;
  const int bk = g.kv_bmod ? b % g.kv_bmod : b;
  const T* k = reinterpret_cast<const T*>(g.k) + (int64_t)bk * g.k_bs + h * dk;
  const T* v = reinterpret_cast<const T*>(g.v) + (int64_t)bk * g.v_bs + h * dk;
  stage_rows<T>(Qs, ldd, q, g.q_ld, Lq, dk, g.temperature, tid);
  stage_rows<T>(Ks, ldd, k, g.k_ld, Lk, dk, 1.f, tid);
  stage_rows<T>(Vs, ldd, v, g.v_ld, Lk, dk, 1.f, tid);
  __syncthreads();

  for (int c = tid; c < Lq * Lk; c += AT_THREADS) {
    int i = c / Lk, j = c % Lk;
    const float* qi = Qs + i * ldd;
    const float* kj = Ks + j * ldd;
    float acc = 0.f;
    for (int d = 0; d < dk; ++d) acc = fmaf(qi[d], kj[d], acc);
    S[i * lds_s + j] = acc;
  }
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
  for (int c = tid; c < Lq * dk; c += AT_THREADS) {
    int i = c / dk, d = c % dk;
    const float* pi = S + i * lds_s;
    float acc = 0.f;
    for (int j = 0; j < Lk; ++j) acc = fmaf(pi[j], Vs[j * ldd + d], acc);
    ob[(int64_t)i * g.o_ld + d] = from_f<T>(acc);
  }
}

template <typename T>
__global__ void __launch_bounds__(AT_THREADS) attn_bwd_kernel(AttnGeom g, const float* __restrict__ probs,
                                                              const T* __restrict__ dout, T* __restrict__ dq,
                                                              T* __restrict__ dkp, T* __restrict__ dvp) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H;
  const int Lq = g.Lq, Lk = g.Lk, dk = g.dk, ldd = dk + 1, lds_s = Lk + 1;
  float* Qs = sm;                 // q / temperature
  float* Ks = Qs + Lq * ldd;
  float* Vs = Ks + Lk * ldd;
  float* dO = Vs + Lk * ldd;
  float* Ps = dO + Lq * ldd;      // p, then dropped p
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

  for (int c = tid; c < Lq * Lk; c += AT_THREADS) {
    int i = c / Lk, j = c % Lk;
    float acc = 0.f;
    for (int d = 0; d < dk; ++d) acc = fmaf(dO[i * ldd + d], Vs[j * ldd + d], acc);
    Ds[i * lds_s + j] = acc;
  }
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
      Ds[i * lds_s + j] = p * (dp - rs);
      Ps[i * lds_s + j] = pd;
    }
  }
  __syncthreads();

  T* dkb = dkp + koff;
  T* dvb = dvp + voff;
  for (int c = tid; c < Lk * dk; c += AT_THREADS) {
    int j = c / dk, d = c % dk;
    float av = 0.f, ak = 0.f;
    for (int i = 0; i < Lq; ++i) {
      av = fmaf(Ps[i * lds_s + j], dO[i * ldd + d], av);
      ak = fmaf(Ds[i * lds_s + j], Qs[i * ldd + d], ak);
    }
    dvb[(int64_t)j * g.v_ld + d] = from_f<T>(av);
    dkb[(int64_t)j * g.k_ld + d] = from_f<T>(ak);
  }
  T* dqb = dq + qoff;
  for (int c = tid; c < Lq * dk; c += AT_THREADS) {
    int i = c / dk, d = c % dk;
    float acc = 0.f;
    for (int j = 0; j < Lk; ++j) acc = fmaf(Ds[i * lds_s + j], Ks[j * ldd + d], acc);
    dqb[(int64_t)i * g.q_ld + d] = from_f<T>(acc / g.temperature);
  }
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

static void check_geom(const AttnGeom& g, DType t) {
  require(g.Lq >= 1 && g.Lq <= 64 && g.Lk >= 1 && g.Lk <= 64, "attention: Lq/Lk must be in [1, 64]");
  require(g.dk % 8 == 0 && g.dk <= 128, "attention: head size must be a multiple of 8 and <= 128");
  (void)t;
}

void attention_fwd(const AttnGeom& g, void* o, float* probs, DType t, hipStream_t s) {
  check_geom(g, t);
  const size_t ldd = g.dk + 1;
  const size_t smem = sizeof(float) * (g.Lq * ldd + 2 * g.Lk * ldd + g.Lq * (g.Lk + 1));
  require(smem <= 160 * 1024, "attention_fwd: LDS budget exceeded");
  dim3 grid(g.B * g.H);
  if (t == DType::F32)
    attn_fwd_kernel<float><<<grid, AT_THREADS, smem, s>>>(g, (float*)o, probs);
  else
    attn_fwd_kernel<bf16><<<grid, AT_THREADS, smem, s>>>(g, (bf16*)o, probs);
  CAPGEN_HIP(hipGetLastError());
}

void attention_bwd(const AttnGeom& g, const float* probs, const void* dout, void* dq, void* dk, void* dv,
                   DType t, hipStream_t s) {
  check_geom(g, t);
  const size_t ldd = g.dk + 1;
  const size_t smem = sizeof(float) * (2 * g.Lq * ldd + 2 * g.Lk * ldd + 2 * g.Lq * (g.Lk + 1));
  require(smem <= 160 * 1024, "attention_bwd: LDS budget exceeded (head size too large)");
  dim3 grid(g.B * g.H);
  if (t == DType::F32)
    attn_bwd_kernel<float><<<grid, AT_THREADS, smem, s>>>(g, probs, (const float*)dout, (float*)dq,
                                                          (float*)dk, (float*)dv);
  else
    attn_bwd_kernel<bf16><<<grid, AT_THREADS, smem, s>>>(g, probs, (const bf16*)dout, (bf16*)dq, (bf16*)dk,
                                                         (bf16*)dv);
  CAPGEN_HIP(hipGetLastError());
}

void attention_head_mean(const float* probs, int B, int H, int Lq, int Lk, int row, float* out, hipStream_t s) {
  int n = B * Lk;
  head_mean_kernel<<<(n + 255) / 256, 256, 0, s>>>(probs, B, H, Lq, Lk, row, out);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
