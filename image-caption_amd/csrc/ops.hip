// capgen — row-wise / elementwise / optimizer kernels for gfx950.
//
// LayerNorm: one wave64 per row (d/64 contiguous elements per lane, 16-B loads), the
// mean/var reductions are cross-lane shuffles; dropout/bias/residual/positional-encoding
// adds and the non-pad row mask are fused in.  Backward accumulates dgamma/dbeta per
// workgroup and issues one f32 atomic per column per workgroup.
// CE: one workgroup per row (V=10000 f32 logits stay in L2 for the 3 passes).
// Adam: 16-B vectorised streaming over the flat parameter arena (HBM bound).
#include <cstdlib>

#include "ops.h"
#include "hazard.h"

namespace capgen {


constexpr int LN_THREADS = 256;  // 4 rows per workgroup
constexpr float LN_EPS = 1e-6f;  // modules.py:57,105


// target of the LayerNorm kernels' absent optional inputs (zeros: residual, bias, positional row)
struct LnDummy {
  float zero[1024];  // the widest row (d = 64 * 16)
  uint64_t seed;
  int32_t id;
  uint8_t valid;
};
__device__ LnDummy g_ln_dummy = {{}, 0, 0, 1};

// Every global load of the row (input, residual, bias, positional row, gamma, beta, row mask,
// dropout seed) is issued before the first store: the kernel pays ONE memory round trip (the
// stores could alias the parameter pointers, so the compiler would not hoist them itself).
template <int DPL>
__device__ __forceinline__ void load_f32(const float* p, float (&out)[DPL]) {
  load_f<float, DPL>(p, out);
}
template <typename T, int DPL>
__global__ void __launch_bounds__(LN_THREADS) ln_fwd_kernel(LnFwd a) {
  StampScope stamp_scope(a.stamp);
  if (a.prio) __builtin_amdgcn_s_setprio(3);
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (LN_THREADS / 64) + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int d = a.d, c0 = lane * DPL;
  const int64_t base = (int64_t)m * d + c0;
  float x[DPL], r[DPL], bias[DPL], pe[DPL], gm[DPL], bt[DPL];
  // optional inputs through a pointer select (absent -> a device dummy of zeros), loaded
  // unconditionally: a load inside a branch is waited for at the branch's join (one more round
  // trip per optional input; the ISA of the branchy form had five)
  // (the uniform base pointers go through opaque() so hipcc cannot turn the select back into a branch)
  const T* res_p = opaque(a.res ? reinterpret_cast<const T*>(a.res) : reinterpret_cast<const T*>(g_ln_dummy.zero)) +
                   (a.res ? base : c0);
  const float* bias_p = opaque(a.a_bias ? a.a_bias : g_ln_dummy.zero) + c0;
  const float* pe_p = opaque(a.pe ? a.pe : g_ln_dummy.zero) + (a.pe ? (int64_t)(m % max(a.pe_L, 1)) * d : 0) + c0;
  const uint64_t* seed_p = opaque(a.drop.seed_ptr ? a.drop.seed_ptr : &g_ln_dummy.seed);
  const int32_t* ids_p = opaque(a.mask.ids ? a.mask.ids : &g_ln_dummy.id) + (a.mask.ids ? (int64_t)m * a.mask.ids_ld : 0);
  const uint8_t* val_p = opaque(a.mask.valid ? a.mask.valid : &g_ln_dummy.valid) + (a.mask.valid ? m : 0);
  const uint64_t seed_v = *seed_p;
  const int idv = *ids_p;
  const int vld = *val_p;
  load_f<T, DPL>(reinterpret_cast<const T*>(a.a) + base, x);
  load_f<T, DPL>(res_p, r);
  load_f32<DPL>(bias_p, bias);
  load_f32<DPL>(pe_p, pe);
  load_f32<DPL>(a.gamma + c0, gm);
  load_f32<DPL>(a.beta + c0, bt);
  const bool kept = !(a.mask.ids && idv == a.mask.pad_idx) && !(a.mask.valid && vld == 0);
  const uint64_t seed = a.drop.seed_ptr ? seed_v : 0;
  if (a.a_bias) {
#pragma unroll
    for (int e = 0; e < DPL; ++e) x[e] += bias[e];
  }
  if (a.drop.seed_ptr) {
#pragma unroll
    for (int e = 0; e < DPL; ++e)
      x[e] = drop_keep(seed, a.drop.site, (uint32_t)(base + e), a.drop.thresh) ? x[e] * a.drop.scale : 0.f;
  }
  if (a.res) {
#pragma unroll
    for (int e = 0; e < DPL; ++e) x[e] += r[e];
  }
  if (a.pe) {
#pragma unroll
    for (int e = 0; e < DPL; ++e) x[e] += pe[e];
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < DPL; ++e) s += x[e];
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < DPL; ++e) {
    float t = x[e] - mean;
    q = fmaf(t, t, q);
  }
  const float var = wave_sum(q) / (float)d;
  const float rstd = 1.0f / sqrtf(var + LN_EPS);
  const float keep = kept ? 1.f : 0.f;
  float y[DPL];
#pragma unroll
  for (int e = 0; e < DPL; ++e) y[e] = ((x[e] - mean) * rstd * gm[e] + bt[e]) * keep;
  bool stored = false;
  if constexpr (DPL * sizeof(T) % 16 == 0) {
    if (a.wt > 0) {  // write-through (capgen_common.h wt_rsrc)
      const uint32_t off = (uint32_t)(base * (int64_t)sizeof(T));
      if (a.v_save) store_wt<T, DPL>(wt_rsrc(a.v_save), off, x);
      store_wt<T, DPL>(wt_rsrc(a.y), off, y);
      stored = true;
    }
  }
  if (!stored) {
    if (a.v_save) store_f<T, DPL>(reinterpret_cast<T*>(a.v_save) + base, x);
    store_f<T, DPL>(reinterpret_cast<T*>(a.y) + base, y);
  }
  if (lane == 0) {
    if (a.mean) a.mean[m] = mean;
    if (a.rstd) a.rstd[m] = rstd;
  }
}

// One row per wave.  The row index is wave-uniform (readfirstlane), so the row statistics, the row
// mask and the dropout seed are scalar loads, issued together with the row's two 16-B vector loads
// (dy, v) and gamma before any use: one memory round trip per row.
//
// (Round 3 ran R = 2 rows per wave -- both rows' loads first -- and, under co-scheduling with the
// side streams, sometimes wrote the row it computed last shifted by a row-scalar-sized amount while
// every input was equal after the call: 12-14 of 30 two-engine comparisons, 0 of 30 at one row.
// Its ISA did not issue the loads together: hipcc drained row 0's dy / v loads with vmcnt(0)
// before loading mean / rstd as per-lane vector loads, then issued row 1's.  The mechanism was not
// isolated; the multi-row variant is deleted, not configured away.)
template <typename T, int DPL, int NT = LN_THREADS>
__global__ void __launch_bounds__(NT) ln_bwd_kernel(LnBwd a) {
  __shared__ float red[3][NT / 64][64 * DPL];
  StampScope stamp_scope(a.stamp);
  if (a.prio) __builtin_amdgcn_s_setprio(3);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int d = a.d, c0 = lane * DPL;
  const int m = blockIdx.x * (NT / 64) + wave;  // wave-uniform
  const bool on = m < a.M;
  const int64_t base = (int64_t)m * d + c0;
  float gm[DPL], dy[DPL], v[DPL];
  float mean = 0.f, rstd = 0.f;
  int idv = 0, vld = 1;
  // optional inputs are read through a pointer select (absent -> a device dummy), never inside a
  // branch: a load in a branch makes hipcc wait for it at the join, one more round trip each
  const uint64_t* seed_p = opaque(a.drop.seed_ptr ? a.drop.seed_ptr : &g_ln_dummy.seed);
  const int32_t* ids_p = opaque(a.mask.ids ? a.mask.ids : &g_ln_dummy.id) +
                         (a.mask.ids ? (int64_t)min(m, a.M - 1) * a.mask.ids_ld : 0);
  const uint8_t* val_p = opaque(a.mask.valid ? a.mask.valid : &g_ln_dummy.valid) + (a.mask.valid ? min(m, a.M - 1) : 0);
  const uint64_t seed_v = *seed_p;
  const int idv_v = *ids_p;
  const int vld_v = *val_p;
  load_f<float, DPL>(a.gamma + c0, gm);
  if (on) {
    load_f<T, DPL>(reinterpret_cast<const T*>(a.dy) + base, dy);
    load_f<T, DPL>(reinterpret_cast<const T*>(a.v) + base, v);
    mean = a.mean[m], rstd = a.rstd[m];
  }
  const uint64_t seed = a.drop.seed_ptr ? seed_v : 0;
  if (a.mask.ids) idv = idv_v;
  if (a.mask.valid) vld = vld_v;
  const bool kept = !(a.mask.ids && idv == a.mask.pad_idx) && vld != 0;
  float dg[DPL], db[DPL], dz[DPL];
#pragma unroll
  for (int e = 0; e < DPL; ++e) dg[e] = db[e] = dz[e] = 0.f;
  if (on) {
    const float keep = kept ? 1.f : 0.f;
    float g[DPL], xh[DPL], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < DPL; ++e) {
      const float y = dy[e] * keep;
      xh[e] = (v[e] - mean) * rstd;
      g[e] = y * gm[e];
      s1 += g[e];
      s2 = fmaf(g[e], xh[e], s2);
      dg[e] = y * xh[e];
      db[e] = y;
    }
    const float mg = wave_sum(s1) / (float)d, mgx = wave_sum(s2) / (float)d;
    float dv[DPL];
#pragma unroll
    for (int e = 0; e < DPL; ++e) dv[e] = rstd * (g[e] - mg - xh[e] * mgx);
    constexpr bool whole = DPL * sizeof(T) % 16 == 0;
    const bool wt = whole && a.wt > 0;
    if (a.d_res) {
      if constexpr (whole) {
        if (wt) store_wt<T, DPL>(wt_rsrc(a.d_res), (uint32_t)(base * (int64_t)sizeof(T)), dv);
        else store_f<T, DPL>(reinterpret_cast<T*>(a.d_res) + base, dv);
      } else {
        store_f<T, DPL>(reinterpret_cast<T*>(a.d_res) + base, dv);
      }
    }
    if (a.d_a) {
      if (a.drop.seed_ptr) {
#pragma unroll
        for (int e = 0; e < DPL; ++e)
          dv[e] = drop_keep(seed, a.drop.site, (uint32_t)(base + e), a.drop.thresh) ? dv[e] * a.drop.scale : 0.f;
      }
      if constexpr (whole) {
        if (wt) store_wt<T, DPL>(wt_rsrc(a.d_a), (uint32_t)(base * (int64_t)sizeof(T)), dv);
        else store_f<T, DPL>(reinterpret_cast<T*>(a.d_a) + base, dv);
      } else {
        store_f<T, DPL>(reinterpret_cast<T*>(a.d_a) + base, dv);
      }
#pragma unroll
      for (int e = 0; e < DPL; ++e) dz[e] = dv[e];
    }
  }
  if (!a.dgamma && !a.dbias) return;
  const int64_t so = (int64_t)(blockIdx.x % a.stripes) * a.stripe_stride;
#pragma unroll
  for (int e = 0; e < DPL; ++e) {
    red[0][wave][c0 + e] = dg[e];
    red[1][wave][c0 + e] = db[e];
    red[2][wave][c0 + e] = dz[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += NT) {
    float sg = 0.f, sb = 0.f, sz = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      sg += red[0][w][c];
      sb += red[1][w][c];
      sz += red[2][w][c];
    }
    if (a.dgamma) {
      atomicAdd(a.dgamma + so + c, sg);
      atomicAdd(a.dbeta + so + c, sb);
    }
    if (a.dbias) atomicAdd(a.dbias + so + c, sz);
  }
}

template <typename T>
static void ln_fwd_dispatch(const LnFwd& a, hipStream_t s) {
  dim3 grid((a.M + 3) / 4);
  switch (a.d / 64) {
    case 1: ln_fwd_kernel<T, 1><<<grid, LN_THREADS, 0, s>>>(a); break;
    case 2: ln_fwd_kernel<T, 2><<<grid, LN_THREADS, 0, s>>>(a); break;
    case 4: ln_fwd_kernel<T, 4><<<grid, LN_THREADS, 0, s>>>(a); break;
    case 8: ln_fwd_kernel<T, 8><<<grid, LN_THREADS, 0, s>>>(a); break;
    case 16: ln_fwd_kernel<T, 16><<<grid, LN_THREADS, 0, s>>>(a); break;
    default: throw Error("layernorm: width must be 64 * {1,2,4,8,16}");
  }
}
void layernorm_fwd(const LnFwd& a_in, DType t, hipStream_t s) {
  if (a_in.M <= 0 || (skip_mask() & 1)) return;
  LnFwd a = a_in;
  if (a.wt < 0) a.wt = wt_default();
  if (hz::active()) {
    using namespace hz;
    const int64_t row = a.d * (int64_t)dsize(t);
    op(s, "ln_fwd", {rd(a.a, a.M * row), rd(a.a_bias, a.d * 4), rd(a.res, a.M * row), rd(a.pe, (int64_t)a.pe_L * a.d * 4),
                     rd(a.gamma, a.d * 4), rd(a.beta, a.d * 4), blk(a.mask.ids, a.M, 4, a.mask.ids_ld * 4, RD),
                     rd(a.mask.valid, a.M), rd(a.drop.seed_ptr, 8), wr(a.y, a.M * row), wr(a.v_save, a.M * row),
                     wr(a.mean, a.M * 4), wr(a.rstd, a.M * 4)});
  }
  if (t == DType::F32) ln_fwd_dispatch<float>(a, s);
  else ln_fwd_dispatch<bf16>(a, s);
  CAPGEN_HIP(hipGetLastError());
}

// 8 rows (waves) per workgroup: half the workgroups -- and half the striped gamma / beta / bias
// atomics -- of the 4-row form (round 5: 2.699-2.703 vs 2.726-2.757 ms/step, three alternating rounds;
// the class 119 vs 137 us/step; 16 rows per workgroup: 2.711-2.716 vs 2.678-2.707 ms, slower)
#ifndef CAPGEN_LNB_NT
#define CAPGEN_LNB_NT 512
#endif
template <typename T, int DPL>
static void ln_bwd_launch(const LnBwd& a, hipStream_t s) {
  // (the per-wave partial sums take 3 * NT * DPL floats of LDS: the widest rows keep 8 waves)
  constexpr int NT = DPL * CAPGEN_LNB_NT > 8 * 1024 ? 512 : CAPGEN_LNB_NT, W = NT / 64;  // one row per wave
  ln_bwd_kernel<T, DPL, NT><<<(a.M + W - 1) / W, NT, 0, s>>>(a);
}
template <typename T>
static void ln_bwd_dispatch(const LnBwd& a, hipStream_t s) {
  switch (a.d / 64) {
    case 1: ln_bwd_launch<T, 1>(a, s); break;
    case 2: ln_bwd_launch<T, 2>(a, s); break;
    case 4: ln_bwd_launch<T, 4>(a, s); break;
    case 8: ln_bwd_launch<T, 8>(a, s); break;
    case 16: ln_bwd_launch<T, 16>(a, s); break;
    default: throw Error("layernorm: width must be 64 * {1,2,4,8,16}");
  }
}
void layernorm_bwd(const LnBwd& a_in, DType t, hipStream_t s) {
  if (a_in.M <= 0 || (skip_mask() & 4)) return;
  LnBwd a = a_in;
  if (a.wt < 0) a.wt = wt_default();
  if (hz::active()) {
    using namespace hz;
    const int64_t row = a.d * (int64_t)dsize(t), sb = a.d * 4, ss = std::max<int64_t>(a.stripe_stride * 4, sb);
    op(s, "ln_bwd", {rd(a.dy, a.M * row), rd(a.v, a.M * row), rd(a.mean, a.M * 4), rd(a.rstd, a.M * 4),
                     rd(a.gamma, a.d * 4), blk(a.mask.ids, a.M, 4, a.mask.ids_ld * 4, RD), rd(a.mask.valid, a.M),
                     rd(a.drop.seed_ptr, 8), wr(a.d_res, a.M * row), wr(a.d_a, a.M * row),
                     blk(a.dgamma, a.stripes, sb, ss, ACC), blk(a.dbeta, a.stripes, sb, ss, ACC),
                     blk(a.dbias, a.stripes, sb, ss, ACC)});
  }
  if (skip_mask() & 128) a.dgamma = a.dbeta = a.dbias = nullptr;  // diagnostic: no parameter-gradient sums
  if (t == DType::F32) ln_bwd_dispatch<float>(a, s);
  else ln_bwd_dispatch<bf16>(a, s);
  CAPGEN_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) pack_kernel(const TI* __restrict__ feats, const float* __restrict__ pos,
                                                   const int32_t* __restrict__ img_idx, int n_img, int N, int F, int P,
                                                   int Kp, int M, TO* __restrict__ out, uint8_t* __restrict__ valid,
                                                   uint64_t* seed_bump) {
  // one wave per row m = (b, n), four rows per workgroup (round 6: the row-per-workgroup form spent its
  // time on a workgroup barrier pair and an LDS atomic per position element; the region flag is now a
  // wave ballot).  Features: 16-B loads, every load of the row issued before its stores.
  constexpr int V = 16 / sizeof(TI);
  const int lane = threadIdx.x & 63, m = blockIdx.x * 4 + (threadIdx.x >> 6);
  // the step's dropout seed advance rides along: nothing in this launch reads the seed
  if (seed_bump && blockIdx.x == 0 && threadIdx.x == 0) *seed_bump += 0x9E3779B97F4A7C15ull;
  if (m >= M) return;  // (whole waves; no workgroup barrier in this kernel)
  // with img_idx the features / positions of image img_idx[b] are read straight from an HBM-resident
  // store (dataset.py:12-18 + DataLoader collate, fused)
  int64_t src = m;
  TO* o = out + (int64_t)m * Kp;
  if (img_idx) {
    const int img = img_idx[m / N];
    if (img < 0 || img >= n_img) {  // out-of-range image: an all-padding row, never an OOB read
      for (int c = lane; c < Kp; c += 64) o[c] = from_f<TO>(0.f);
      if (lane == 0) valid[m] = 0;
      return;
    }
    src = (int64_t)img * N + m % N;
  }
  const TI* f = feats + src * F;
  const float* p = pos + src * P;
  typedef typename Vec16<TI>::type VT;
  constexpr int U = 4;  // 16-B loads in flight per lane
  for (int c0 = lane * V; c0 < F; c0 += 64 * V * U) {
    VT v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * 64 * V;
      if (c < F) v[u] = *reinterpret_cast<const VT*>(f + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = c0 + u * 64 * V;
      if (c >= F) break;
      const TI* e = reinterpret_cast<const TI*>(&v[u]);
      float x[V];
#pragma unroll
      for (int j = 0; j < V; ++j) x[j] = to_f(e[j]);
      store_f<TO, V>(o + c, x);
    }
  }
  // positions, then zeros to Kp; a region is padding iff its position row is all zero (model.py:206)
  bool nz = false;
  for (int c = F + lane; c < Kp; c += 64) {
    float x = 0.f;
    if (c < F + P) {
      x = p[c - F];
      nz |= x != 0.f;
    }
    o[c] = from_f<TO>(x);
  }
  const bool any = __ballot(nz) != 0;
  if (lane == 0) valid[m] = any ? 1 : 0;
}

void pack_encoder_input(const void* feats, DType ft, const float* pos, int M, int F, int P, int Kp, void* out,
                        DType ot, uint8_t* valid, hipStream_t s, const int32_t* img_idx, int N, int n_img,
                        uint64_t* seed_bump) {
  if (M <= 0) return;
  require(F % 8 == 0 && ((uintptr_t)feats & 15) == 0, "pack: feature width must be a multiple of 8, 16-B aligned");
  require(img_idx == nullptr || N > 0, "pack: indexed gather needs N");
  if (hz::active()) {
    using namespace hz;
    const int64_t src_rows = img_idx ? (int64_t)n_img * N : M;
    op(s, "pack", {rd(feats, src_rows * F * (int64_t)dsize(ft)), rd(pos, src_rows * P * 4), rd(img_idx, img_idx ? M / N * 4 : 0),
                   wr(out, (int64_t)M * Kp * dsize(ot)), wr(valid, M), wr(seed_bump, 8)});
  }
  dim3 grid((M + 3) / 4);
  if (ft == DType::F32 && ot == DType::F32)
    pack_kernel<float, float><<<grid, 256, 0, s>>>((const float*)feats, pos, img_idx, n_img, N, F, P, Kp, M, (float*)out, valid, seed_bump);
  else if (ft == DType::F32 && ot == DType::BF16)
    pack_kernel<float, bf16><<<grid, 256, 0, s>>>((const float*)feats, pos, img_idx, n_img, N, F, P, Kp, M, (bf16*)out, valid, seed_bump);
  else if (ft == DType::BF16 && ot == DType::BF16)
    pack_kernel<bf16, bf16><<<grid, 256, 0, s>>>((const bf16*)feats, pos, img_idx, n_img, N, F, P, Kp, M, (bf16*)out, valid, seed_bump);
  else
    pack_kernel<bf16, float><<<grid, 256, 0, s>>>((const bf16*)feats, pos, img_idx, n_img, N, F, P, Kp, M, (float*)out, valid, seed_bump);
  CAPGEN_HIP(hipGetLastError());
}

__global__ void prep_caps_kernel(const int32_t* __restrict__ caps, int B, int T, int pad, int32_t* ids_in,
                                 int32_t* tgt, float* count, uint64_t* seed_bump, float* inv_count) {
  __shared__ int cnt;
  if (threadIdx.x == 0) cnt = 0;
  // the step's dropout seed advance (bump_seed) rides along: no kernel in this launch reads it
  if (seed_bump && threadIdx.x == 0) *seed_bump += 0x9E3779B97F4A7C15ull;
  __syncthreads();
  const int L = T - 1;
  int local = 0;
  for (int c = threadIdx.x; c < B * L; c += blockDim.x) {
    int b = c / L, t = c % L;
    ids_in[c] = caps[b * T + t];
    int y = caps[b * T + t + 1];
    tgt[c] = y;
    local += (y != pad);
  }
  atomicAdd(&cnt, local);
  __syncthreads();
  if (threadIdx.x == 0) *count = (float)cnt;
  if (inv_count && threadIdx.x == 0) *inv_count = 1.f / (float)cnt;  // as loss_finalize's 1.f / n
}

void prepare_captions(const int32_t* caps, int B, int T, int pad, int32_t* ids_in, int32_t* tgt, float* count,
                      hipStream_t s, uint64_t* seed_bump, float* inv_count) {
  if (hz::active()) {
    using namespace hz;
    op(s, "prep_captions", {rd(caps, (int64_t)B * T * 4), wr(ids_in, (int64_t)B * (T - 1) * 4),
                            wr(tgt, (int64_t)B * (T - 1) * 4), wr(count, 4), wr(seed_bump, 8), wr(inv_count, 4)});
  }
  prep_caps_kernel<<<1, 1024, 0, s>>>(caps, B, T, pad, ids_in, tgt, count, seed_bump, inv_count);
  CAPGEN_HIP(hipGetLastError());
}

template <typename T>
__global__ void gather_kernel(const float* __restrict__ table, const int32_t* __restrict__ ids, int64_t ids_ld,
                              int M, int d, T* __restrict__ out) {
  int64_t n = (int64_t)M * d;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
    int64_t m = c / d;
    int col = c % d;
    out[c] = from_f<T>(table[(int64_t)ids[m * ids_ld] * d + col]);
  }
}
void embedding_gather(const float* table, const int32_t* ids, int64_t ids_ld, int M, int d, void* out, DType t,
                      hipStream_t s, int64_t table_rows) {
  if (M <= 0) return;
  if (hz::active())
    hz::op(s, "emb_gather", {hz::rd(table, table_rows * d * 4), hz::blk(ids, M, 4, ids_ld * 4, hz::RD),
                             hz::wr(out, (int64_t)M * d * dsize(t))});
  int64_t n = (int64_t)M * d;
  int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  if (t == DType::F32) gather_kernel<float><<<grid, 256, 0, s>>>(table, ids, ids_ld, M, d, (float*)out);
  else gather_kernel<bf16><<<grid, 256, 0, s>>>(table, ids, ids_ld, M, d, (bf16*)out);
  CAPGEN_HIP(hipGetLastError());
}

template <typename T>
__global__ void scatter_kernel(const T* __restrict__ dE, const int32_t* __restrict__ ids, int M, int d, int pad,
                               float* __restrict__ grad) {
  int64_t n = (int64_t)M * d;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < n; c += (int64_t)gridDim.x * blockDim.x) {
    int64_t m = c / d;
    int id = ids[m];
    if (id == pad) continue;
    atomicAdd(grad + (int64_t)id * d + (c % d), to_f(dE[c]));
  }
}
void embedding_scatter_add(const void* dE, const int32_t* ids, int M, int d, int pad, float* grad, DType t,
                           hipStream_t s, int64_t table_rows) {
  if (M <= 0) return;
  if (hz::active())
    hz::op(s, "emb_scatter", {hz::rd(dE, (int64_t)M * d * dsize(t)), hz::rd(ids, (int64_t)M * 4),
                              hz::acc(grad, table_rows * d * 4)});
  int64_t n = (int64_t)M * d;
  int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  if (t == DType::F32) scatter_kernel<float><<<grid, 256, 0, s>>>((const float*)dE, ids, M, d, pad, grad);
  else scatter_kernel<bf16><<<grid, 256, 0, s>>>((const bf16*)dE, ids, M, d, pad, grad);
  CAPGEN_HIP(hipGetLastError());
}

// db[n] += alpha * sum_m X[m][n]: 16-B loads (a workgroup covers 8 vectors x 32 row lanes x
// 8 rows per lane), rows reduced through LDS, one atomic per column per workgroup
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ X, int M, int N, int64_t ldx, float alpha,
                                                     const float* alpha_ptr, float* __restrict__ db, int stripes,
                                                     int64_t stripe_stride) {
  constexpr int V = 16 / sizeof(T);
  __shared__ float red[32][8 * V + 1];
  const int cv = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int n = (blockIdx.x * 8 + cv) * V;
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  if (n < N) {
    const int r0 = blockIdx.y * 256;
#pragma unroll 4
    for (int j = 0; j < 8; ++j) {
      const int m = r0 + rl + 32 * j;
      if (m < M) {
        float x[V];
        load_f<T, V>(X + (int64_t)m * ldx + n, x);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += x[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) red[rl][cv * V + e] = acc[e];
  __syncthreads();
  if (threadIdx.x < 8 * V) {
    const int c = threadIdx.x;
    const int nn = blockIdx.x * 8 * V + c;
    if (nn < N) {
      float sum = 0.f;
      for (int r = 0; r < 32; ++r) sum += red[r][c];
      const float a = alpha_ptr ? alpha * *alpha_ptr : alpha;
      atomicAdd(db + (int64_t)(blockIdx.y % stripes) * stripe_stride + nn, a * sum);
    }
  }
}
void column_sum(const void* X, int M, int N, int64_t ldx, float alpha, const float* alpha_ptr, float* db, DType t,
                hipStream_t s, int stripes, int64_t stripe_stride) {
  if (M <= 0 || N <= 0) return;
  const int V = t == DType::F32 ? 4 : 8;
  require(N % V == 0 && ldx % V == 0, "column_sum: N/ld must be multiples of 16 B");
  if (hz::active()) {
    using namespace hz;
    op(s, "column_sum", {blk(X, M, N * (int64_t)dsize(t), ldx * (int64_t)dsize(t), RD), rd(alpha_ptr, 4),
                         blk(db, stripes, N * 4, std::max<int64_t>(stripe_stride * 4, N * 4), ACC)});
  }
  dim3 grid((N + 8 * V - 1) / (8 * V), (M + 255) / 256);
  if (t == DType::F32) colsum_kernel<float><<<grid, 256, 0, s>>>((const float*)X, M, N, ldx, alpha, alpha_ptr, db, stripes,
                                                               stripe_stride);
  else colsum_kernel<bf16><<<grid, 256, 0, s>>>((const bf16*)X, M, N, ldx, alpha, alpha_ptr, db, stripes,
                                                              stripe_stride);
  CAPGEN_HIP(hipGetLastError());
}

__global__ void stripe_reduce_kernel(float* __restrict__ S, int stripes, int64_t stride, int64_t n,
                                     float* __restrict__ dst, int accumulate, int clear) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float acc = accumulate ? dst[i] : 0.f;
    for (int k = 0; k < stripes; ++k) acc += S[k * stride + i];
    dst[i] = acc;
    if (clear)
      for (int k = 0; k < stripes; ++k) S[k * stride + i] = 0.f;
  }
}
void stripe_reduce(float* S, int stripes, int64_t stride, int64_t n, float* dst, int accumulate, hipStream_t s,
                   int clear) {
  if (n <= 0) return;
  if (hz::active()) {
    using namespace hz;
    const int64_t ss = std::max<int64_t>(stride * 4, n * 4);
    op(s, "stripe_reduce", {blk(S, stripes, n * 4, ss, clear ? WR : RD), blk(S, stripes, n * 4, ss, RD), wr(dst, n * 4),
                            accumulate ? rd(dst, n * 4) : Rgn{}});
  }
  int grid = (int)std::min<int64_t>((n + 255) / 256, 1024);
  stripe_reduce_kernel<<<grid, 256, 0, s>>>(S, stripes, stride, n, dst, accumulate, clear);
  CAPGEN_HIP(hipGetLastError());
}

// ---- block reductions (256 threads = 4 waves) ----
__device__ __forceinline__ float block_max(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();
  return r;
}

template <typename T>
__global__ void __launch_bounds__(256) ce_kernel(const float* __restrict__ logits, const int32_t* __restrict__ tgt,
                                                 int V, int pad, float* __restrict__ loss_row, T* __restrict__ dl) {
  __shared__ float sh[4];
  const int m = blockIdx.x;
  const float* x = logits + (int64_t)m * V;
  T* g = dl + (int64_t)m * V;
  const int y = tgt[m];
  if (y == pad) {
    for (int c = threadIdx.x; c < V; c += 256) g[c] = from_f<T>(0.f);
    if (threadIdx.x == 0) loss_row[m] = 0.f;
    return;
  }
  float mx = -INFINITY;
  for (int c = threadIdx.x; c < V; c += 256) mx = fmaxf(mx, x[c]);
  mx = block_max(mx, sh);
  float se = 0.f;
  for (int c = threadIdx.x; c < V; c += 256) se += expf(x[c] - mx);
  se = block_sum(se, sh);
  const float inv = 1.f / se;
  for (int c = threadIdx.x; c < V; c += 256) {
    float p = expf(x[c] - mx) * inv;
    g[c] = from_f<T>(p - (c == y ? 1.f : 0.f));
  }
  if (threadIdx.x == 0) loss_row[m] = (logf(se) + mx) - x[y];
}
// Register-resident variant (V % 4 == 0, V <= 1024 * NV4): the row is loaded ONCE as float4s
// (every load in flight together: one memory round trip instead of three dependent passes),
// max / sum-exp / gradient are computed from registers.
template <typename T, int NV4>
__global__ void __launch_bounds__(256) ce_reg_kernel(const float* __restrict__ logits, const int32_t* __restrict__ tgt,
                                                     int V, int pad, float* __restrict__ loss_row, T* __restrict__ dl) {
  __shared__ float sh[4];
  const int m = blockIdx.x, V4 = V >> 2;
  const float4* x = reinterpret_cast<const float4*>(logits + (int64_t)m * V);
  T* g = dl + (int64_t)m * V;
  const int y = tgt[m];
  if (y == pad) {
    for (int c = threadIdx.x; c < V; c += 256) g[c] = from_f<T>(0.f);
    if (threadIdx.x == 0) loss_row[m] = 0.f;
    return;
  }
  float4 v[NV4];
  float mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < NV4; ++u) {
    const int c4 = threadIdx.x + 256 * u;
    v[u] = c4 < V4 ? x[c4] : float4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  }
#pragma unroll
  for (int u = 0; u < NV4; ++u) mx = fmaxf(mx, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
  mx = block_max(mx, sh);
  float se = 0.f;
#pragma unroll
  for (int u = 0; u < NV4; ++u) {
    v[u].x = expf(v[u].x - mx), v[u].y = expf(v[u].y - mx), v[u].z = expf(v[u].z - mx), v[u].w = expf(v[u].w - mx);
    se += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  se = block_sum(se, sh);
  const float inv = 1.f / se;
#pragma unroll
  for (int u = 0; u < NV4; ++u) {
    const int c4 = threadIdx.x + 256 * u;
    if (c4 >= V4) continue;
    const int c = 4 * c4;
    float o[4] = {v[u].x * inv, v[u].y * inv, v[u].z * inv, v[u].w * inv};
    if (y >= c && y < c + 4) o[y - c] -= 1.f;
    store_f<T, 4>(g + c, o);
  }
  if (threadIdx.x == 0) loss_row[m] = (logf(se) + mx) - logits[(int64_t)m * V + y];
}

template <typename T>
static void ce_launch(const float* logits, const int32_t* tgt, int M, int V, int pad, float* loss_row, T* dl,
                      hipStream_t s) {
  if (V % 4 == 0 && V <= 1024 * 16) {
    const int nv4 = (V / 4 + 255) / 256;
    if (nv4 <= 4) ce_reg_kernel<T, 4><<<M, 256, 0, s>>>(logits, tgt, V, pad, loss_row, dl);
    else if (nv4 <= 8) ce_reg_kernel<T, 8><<<M, 256, 0, s>>>(logits, tgt, V, pad, loss_row, dl);
    else if (nv4 <= 10) ce_reg_kernel<T, 10><<<M, 256, 0, s>>>(logits, tgt, V, pad, loss_row, dl);
    else ce_reg_kernel<T, 16><<<M, 256, 0, s>>>(logits, tgt, V, pad, loss_row, dl);
  } else {
    ce_kernel<T><<<M, 256, 0, s>>>(logits, tgt, V, pad, loss_row, dl);
  }
}
void cross_entropy_rows(const float* logits, const int32_t* tgt, int M, int V, int pad, float* loss_row, void* dl,
                        DType t, hipStream_t s) {
  if (M <= 0) return;
  if (hz::active())
    hz::op(s, "cross_entropy", {hz::rd(logits, (int64_t)M * V * 4), hz::rd(tgt, (int64_t)M * 4),
                                hz::wr(loss_row, (int64_t)M * 4), hz::wr(dl, (int64_t)M * V * dsize(t))});
  if (t == DType::F32) ce_launch<float>(logits, tgt, M, V, pad, loss_row, (float*)dl, s);
  else ce_launch<bf16>(logits, tgt, M, V, pad, loss_row, (bf16*)dl, s);
  CAPGEN_HIP(hipGetLastError());
}

// Second half of the fused classifier + cross entropy (GemmArgs::ce_stats): the classifier GEMM
// left e = exp(v - mx_c) in bf16 and {mx_c, s_c} per 16-column slab c of each row.  One
// workgroup per row: lse = M + log sum_c s_c exp(mx_c - M), loss_row = lse - v[tgt], and the
// row is rewritten in place as softmax - onehot = e * exp(mx_c - lse) - onehot.  Every load of the
// row (stats + the thread's slabs) is issued up front: one memory round trip.
template <int SPT, int VW>
__global__ void __launch_bounds__(256) ce_finish_kernel(const float2* __restrict__ stats, int64_t ld,
                                                        const float* __restrict__ tlogit,
                                                        const int32_t* __restrict__ tgt, int V, int pad,
                                                        float* __restrict__ loss_row, bf16* __restrict__ dl) {
  // VW = elements per access: 8 (16-B loads / stores, rows 16-B aligned: V % 8 == 0) or 4
  __shared__ float sh[4];
  typedef __attribute__((ext_vector_type(VW))) __bf16 bv;
  constexpr int NQ = 16 / VW;  // accesses per 16-column slab
  const int m = blockIdx.x, nsl = (V + 15) / 16;
  bf16* row = dl + (int64_t)m * V;
  // every load first -- target, target logit, slab stats, the row's e values -- from clamped in-range
  // addresses with no branch around them (a load in a branch is waited for at its join): one round trip
  const int y = tgt[m];
  const float tl = tlogit[m];
  float2 st[SPT];
  bv e[SPT][NQ];
#pragma unroll
  for (int u = 0; u < SPT; ++u) {
    const int c = threadIdx.x + 256 * u, cc = min(c, nsl - 1);
    st[u] = stats[(int64_t)m * ld + cc];
#pragma unroll
    for (int q = 0; q < NQ; ++q) e[u][q] = *reinterpret_cast<const bv*>(row + min(cc * 16 + q * VW, V - VW));
  }
#pragma unroll
  for (int u = 0; u < SPT; ++u)
    if (threadIdx.x + 256 * u >= nsl) st[u] = float2{-INFINITY, 0.f};
  if (y == pad) {  // (uniform per workgroup)
    for (int c = threadIdx.x * VW; c < V; c += 256 * VW) *reinterpret_cast<bv*>(row + c) = bv{};
    if (threadIdx.x == 0) loss_row[m] = 0.f;
    return;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < SPT; ++u) mx = fmaxf(mx, st[u].x);
  mx = block_max(mx, sh);
  float se = 0.f;
#pragma unroll
  for (int u = 0; u < SPT; ++u) se += st[u].y == 0.f ? 0.f : st[u].y * expf(st[u].x - mx);
  se = block_sum(se, sh);
  const float lse = mx + logf(se);
#pragma unroll
  for (int u = 0; u < SPT; ++u) {
    const int c = threadIdx.x + 256 * u;
    if (c >= nsl) continue;
    const float f = expf(st[u].x - lse);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int col = c * 16 + q * VW;
      if (col >= V) continue;
      bv o;
#pragma unroll
      for (int i = 0; i < VW; ++i) {
        float x = (float)e[u][q][i] * f;
        if (y == col + i) x -= 1.f;
        o[i] = (bf16)x;
      }
      *reinterpret_cast<bv*>(row + col) = o;
    }
  }
  if (threadIdx.x == 0) loss_row[m] = lse - tl;
}
void ce_finish(const float2* stats, int64_t ld, const float* tlogit, const int32_t* tgt, int M, int V, int pad,
               float* loss_row, bf16* dl, hipStream_t s) {
  if (M <= 0) return;
  require(V % 4 == 0 && ld >= (V + 15) / 16, "ce_finish: V must be a multiple of 4");
  if (hz::active()) {
    using namespace hz;
    op(s, "ce_finish", {blk(stats, M, (int64_t)((V + 15) / 16) * 8, ld * 8, RD), rd(tlogit, (int64_t)M * 4),
                        rd(tgt, (int64_t)M * 4), wr(loss_row, (int64_t)M * 4), wr(dl, (int64_t)M * V * 2)});
  }
  const int spt = ((V + 15) / 16 + 255) / 256;
  // 16-B accesses when every row starts 16-B aligned (Knob::CeVec8 = 0: the 8-B form, bit-identity test)
  const bool v8 = knob(Knob::CeVec8) != 0 && V % 8 == 0 && ((uintptr_t)dl & 15) == 0;
  auto go = [&](auto spt_c) {
    constexpr int S = decltype(spt_c)::value;
    if (v8) ce_finish_kernel<S, 8><<<M, 256, 0, s>>>(stats, ld, tlogit, tgt, V, pad, loss_row, dl);
    else ce_finish_kernel<S, 4><<<M, 256, 0, s>>>(stats, ld, tlogit, tgt, V, pad, loss_row, dl);
  };
  if (spt <= 1) go(std::integral_constant<int, 1>{});
  else if (spt <= 2) go(std::integral_constant<int, 2>{});
  else if (spt <= 3) go(std::integral_constant<int, 3>{});
  else if (spt <= 4) go(std::integral_constant<int, 4>{});
  else if (spt <= 8) go(std::integral_constant<int, 8>{});
  else throw Error("ce_finish: V > 32768");
  CAPGEN_HIP(hipGetLastError());
}

// CE mean over the (global) non-pad count and the FocalLoss transform (model.py:73-76,
// loss.py:20-28, gamma = 2, applied to the already-averaged CE).  ce_in != null: the mean CE is
// given (the data-parallel path all-reduces the per-rank partial sums first); partial: only
// the per-rank partial mean sum(rows) / count is written to loss_out.
__global__ void loss_finalize_kernel(const float* __restrict__ loss_row, int M, const float* count, int focal,
                                     const float* ce_in, int partial, float* loss_out, float* grad_scale) {
  __shared__ float sh[4];
  float acc = 0.f;
  if (!ce_in)
    for (int c = threadIdx.x; c < M; c += 256) acc += loss_row[c];
  acc = block_sum(acc, sh);
  if (threadIdx.x == 0) {
    const float n = *count;
    const float ce = ce_in ? *ce_in : acc / n;
    if (partial) {
      *loss_out = ce;
    } else if (focal) {
      const float pt = expf(-ce);
      const float om = 1.f - pt;
      *loss_out = om * om * ce;
      if (grad_scale) *grad_scale = (2.f * om * pt * ce + om * om) / n;
    } else {
      *loss_out = ce;
      if (grad_scale) *grad_scale = 1.f / n;
    }
  }
}
void loss_finalize(const float* loss_row, int M, const float* count, int focal, float* loss_out, float* grad_scale,
                   hipStream_t s, const float* ce_in, int partial) {
  if (hz::active())
    hz::op(s, "loss_finalize", {hz::rd(ce_in ? nullptr : loss_row, (int64_t)M * 4), hz::rd(count, 4), hz::rd(ce_in, 4),
                                hz::wr(loss_out, 4), hz::wr(partial ? nullptr : grad_scale, 4)});
  loss_finalize_kernel<<<1, 256, 0, s>>>(loss_row, M, count, focal, ce_in, partial, loss_out, grad_scale);
  CAPGEN_HIP(hipGetLastError());
}

// ---- Adam ---------------------------------------------------------------------------
__global__ void adam_prep_kernel(int64_t* step, float lr, float b1, float b2, float* scal) {
  const int64_t t = ++(*step);
  const double bc1 = 1.0 - pow((double)b1, (double)t);
  const double bc2 = 1.0 - pow((double)b2, (double)t);
  scal[0] = (float)(-(double)lr / bc1);  // value of addcdiv_ (= -step_size)
  scal[1] = (float)sqrt(bc2);            // bias_correction2_sqrt
}
void adam_prepare(int64_t* step, float lr, float b1, float b2, float* scal, hipStream_t s) {
  if (hz::active()) hz::op(s, "adam_prepare", {hz::wr(step, 8), hz::wr(scal, 8)});
  adam_prep_kernel<<<1, 1, 0, s>>>(step, lr, b1, b2, scal);
  CAPGEN_HIP(hipGetLastError());
}


// Adam streams 30 B per parameter that nothing else in the step reads (f32 params, grads, moments:
// 16 B in, 12 B out) beside the critical chain, so (a) those streams use non-temporal loads and
// stores -- they should not push the chain's GEMM panels out of the L2 / Infinity Cache -- while the
// bf16 shadow and the tiled copies, which the next forward reads, keep the default policy; and (b)
// every thread keeps ADAM_U 16-B loads of each array in flight (4 x ADAM_U loads issued before the
// first use), so one workgroup per CU moves the stream at a useful rate (one load per array per
// iteration measured 3.1 TB/s, round 4).
constexpr int ADAM_U = 4;
typedef float adam_f4 __attribute__((ext_vector_type(4)));  // (the nontemporal builtins take clang vectors)
__global__ void __launch_bounds__(256) adam_kernel(adam_f4* __restrict__ p, const adam_f4* __restrict__ g,
                                                   adam_f4* __restrict__ m, adam_f4* __restrict__ v, size_t n4,
                                                   float b1, float b2, float eps, const float* __restrict__ scal,
                                                   bf16* __restrict__ shadow, size_t n_shadow, AdamTiles tiles) {
  const float neg_step = scal[0], bc2s = scal[1];
  const float b1c = 1.f - b1, b2c = 1.f - b2;
  const size_t stride = (size_t)gridDim.x * 256 * ADAM_U;
  for (size_t base = blockIdx.x * (size_t)(256 * ADAM_U) + threadIdx.x; base < n4; base += stride) {
    adam_f4 pp[ADAM_U], gg[ADAM_U], mm[ADAM_U], vv[ADAM_U];
#pragma unroll
    for (int u = 0; u < ADAM_U; ++u) {
      // (a lane past the end re-reads element base: in range, its results are not stored)
      const size_t i = base + (size_t)u * 256 < n4 ? base + (size_t)u * 256 : base;
      pp[u] = __builtin_nontemporal_load(p + i);
      gg[u] = __builtin_nontemporal_load(g + i);
      mm[u] = __builtin_nontemporal_load(m + i);
      vv[u] = __builtin_nontemporal_load(v + i);
    }
    // every load above is issued before the first value is consumed (hipcc otherwise sinks each
    // group of loads to its use, leaving one array's load in flight at a time)
#pragma unroll
    for (int u = 0; u < ADAM_U; ++u) asm volatile("" : "+v"(pp[u]), "+v"(gg[u]), "+v"(mm[u]), "+v"(vv[u]));
#pragma unroll
    for (int u = 0; u < ADAM_U; ++u) {
      const size_t i = base + (size_t)u * 256;
      if (i >= n4) break;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float pc = pp[u][c], mc = mm[u][c], vc = vv[u][c];
        adam_one(pc, gg[u][c], mc, vc, b1c, b2, b2c, eps, neg_step, bc2s);
        pp[u][c] = pc, mm[u][c] = mc, vv[u][c] = vc;
      }
      __builtin_nontemporal_store(pp[u], p + i);
      __builtin_nontemporal_store(mm[u], m + i);
      __builtin_nontemporal_store(vv[u], v + i);
      if (shadow && 4 * i < n_shadow) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 o = {(bf16)pp[u][0], (bf16)pp[u][1], (bf16)pp[u][2], (bf16)pp[u][3]};
        *reinterpret_cast<bf16x4*>(shadow + 4 * i) = o;
        // the fused attention fronts' tiled copy (qkv_tile_weights layout): 4 consecutive k of one
        // row land in one 8-B piece of the row's 16-B fragment slot
#pragma unroll
        for (int t = 0; t < AdamTiles::kMax; ++t) {
          const int64_t rel = (int64_t)(4 * i) - tiles.off[t];
          if (t < tiles.n && rel >= 0 && rel < tiles.len[t]) {
            const int64_t row = rel >> 9;
            const int k = (int)(rel & 511);
            const int64_t piece = (((row >> 4) * 16 + (k >> 5)) * 64 + (row & 15) + 16 * ((k >> 3) & 3)) * 8 + (k & 7);
            *reinterpret_cast<bf16x4*>(tiles.dst[t] + piece) = o;
          }
        }
      }
    }
  }
}
void adam_update(float* p, const float* g, float* m, float* v, size_t n, float b1, float b2, float eps,
                 const float* scal, bf16* shadow, size_t n_shadow, hipStream_t s, int grid_cap,
                 const AdamTiles& tiles) {
  require(tiles.n >= 0 && tiles.n <= AdamTiles::kMax, "adam: at most kMax tiled ranges");
  for (int t = 0; t < tiles.n; ++t)
    // (the tile formula needs only the element offset from the matrix start; 4-aligned so a thread's
    // 4 elements stay in one row)
    require(shadow && tiles.off[t] % 4 == 0 && tiles.len[t] % (16 * 512) == 0 && tiles.off[t] >= 0 &&
                tiles.off[t] + tiles.len[t] <= (int64_t)n_shadow && tiles.dst[t],
            "adam: a tiled range must be whole 16-row blocks of 512-wide rows inside the shadow range");
  require(n % 4 == 0 && n_shadow % 4 == 0, "adam: arena size must be a multiple of 4");
  if (skip_mask() & 32) return;
  if (hz::active())
    hz::op(s, "adam", {hz::rd(g, (int64_t)n * 4), hz::rd(scal, 8), hz::wr(p, (int64_t)n * 4), hz::wr(m, (int64_t)n * 4),
                       hz::wr(v, (int64_t)n * 4), hz::wr(shadow, (int64_t)n_shadow * 2),
                       hz::wr(tiles.n > 0 ? tiles.dst[0] : nullptr, tiles.n > 0 ? tiles.len[0] * 2 : 0),
                       hz::wr(tiles.n > 1 ? tiles.dst[1] : nullptr, tiles.n > 1 ? tiles.len[1] * 2 : 0),
                       hz::wr(tiles.n > 2 ? tiles.dst[2] : nullptr, tiles.n > 2 ? tiles.len[2] * 2 : 0),
                       hz::wr(tiles.n > 3 ? tiles.dst[3] : nullptr, tiles.n > 3 ? tiles.len[3] * 2 : 0)});
  size_t n4 = n / 4;
  // Adam workgroups (grid-stride): one per CU leaves the other wave slots to the critical stream
  // (A/B over 4 runs each: 3.046 vs 3.070 ms/step with 8 per CU)
  constexpr int cap = 256;
  // grid_cap > 0: the caller's cap (an update on the step's critical path takes the whole chip)
  int grid = (int)std::min<size_t>((n4 + 256 * ADAM_U - 1) / (256 * ADAM_U), (size_t)(grid_cap > 0 ? grid_cap : cap));
  adam_kernel<<<grid, 256, 0, s>>>((adam_f4*)p, (const adam_f4*)g, (adam_f4*)m, (adam_f4*)v, n4, b1, b2, eps, scal,
                                   shadow, n_shadow, tiles);
  CAPGEN_HIP(hipGetLastError());
}

// Position-weighted sum of the f32 bit patterns, sum_i bits(x_i) * (2 i + 1) mod 2^64: exact and
// independent of summation order, so equal arenas give equal values on every rank / run.
__global__ void checksum_kernel(const uint32_t* __restrict__ x, size_t n, unsigned long long* out) {
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += (unsigned long long)x[i] * (2ull * i + 1ull);
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}
uint64_t arena_checksum(const float* p, size_t n, hipStream_t s) {
  unsigned long long* d = nullptr;
  CAPGEN_HIP(hipMalloc(&d, sizeof *d));
  CAPGEN_HIP(hipMemsetAsync(d, 0, sizeof *d, s));
  checksum_kernel<<<1024, 256, 0, s>>>(reinterpret_cast<const uint32_t*>(p), n, d);
  CAPGEN_HIP(hipGetLastError());
  unsigned long long v = 0;
  CAPGEN_HIP(hipMemcpyAsync(&v, d, sizeof v, hipMemcpyDeviceToHost, s));
  CAPGEN_HIP(hipStreamSynchronize(s));
  CAPGEN_HIP(hipFree(d));
  return v;
}

__global__ void to_bf16_kernel(const float* __restrict__ src, bf16* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = (bf16)src[i];
}
// 4 elements per lane: one dwordx4 load, one 8-byte store (the sharded update's shadow re-cast)
__global__ void to_bf16x4_kernel(const float4* __restrict__ src, bf16* __restrict__ dst, size_t n4) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 x = src[i];
    bf16x4 o = {(bf16)x.x, (bf16)x.y, (bf16)x.z, (bf16)x.w};
    *reinterpret_cast<bf16x4*>(dst + 4 * i) = o;
  }
}
void to_bf16(const float* src, bf16* dst, size_t n, hipStream_t s) {
  if (!n) return;
  if (hz::active()) hz::op(s, "to_bf16", {hz::rd(src, (int64_t)n * 4), hz::wr(dst, (int64_t)n * 2)});
  if (n % 4 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 7) == 0) {
    const size_t n4 = n / 4;
    int grid = (int)std::min<size_t>((n4 + 255) / 256, 2048);
    to_bf16x4_kernel<<<grid, 256, 0, s>>>((const float4*)src, dst, n4);
    CAPGEN_HIP(hipGetLastError());
    return;
  }
  int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
  to_bf16_kernel<<<grid, 256, 0, s>>>(src, dst, n);
  CAPGEN_HIP(hipGetLastError());
}

// ---- greedy / beam helpers ---------------------------------------------------------
// logsm = 0: argmax of Softmax (Transformer, model.py:124-128); 1: of LogSoftmax
// (PolicyNetwork, model_RL.py:72,126-127) -- the same token except where the rounding of the
// two scores makes different near-ties
// NV > 0: the row (V <= 256 NV) is read once into registers, every load up front (one memory
// round trip instead of three dependent passes); the same per-thread order as the NV = 0 loops
template <int NV>
__global__ void __launch_bounds__(256) argmax_softmax_kernel(const float* __restrict__ logits, int V,
                                                             int64_t* ids_out, int64_t ids_ld, int col,
                                                             int32_t* next_ids, int64_t next_ld, int logsm) {
  __shared__ float sh[4];
  __shared__ float bv[4];
  __shared__ int bi[4];
  const int b = blockIdx.x;
  const float* x = logits + (int64_t)b * V;
  float xr[NV > 0 ? NV : 1];
  float mx = -INFINITY;
  if constexpr (NV > 0) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int c = threadIdx.x + 256 * u;
      xr[u] = c < V ? x[c] : -INFINITY;
      mx = fmaxf(mx, xr[u]);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) mx = fmaxf(mx, x[c]);
  }
  mx = block_max(mx, sh);
  float se = 0.f;
  if constexpr (NV > 0) {
#pragma unroll
    for (int u = 0; u < NV; ++u)
      if (threadIdx.x + 256 * u < V) se += expf(xr[u] - mx);
  } else {
    for (int c = threadIdx.x; c < V; c += 256) se += expf(x[c] - mx);
  }
  se = block_sum(se, sh);
  // argmax over the softmax probabilities, first index on ties (torch.argmax)
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  const float lse = logf(se);
  if constexpr (NV > 0) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int c = threadIdx.x + 256 * u;
      if (c < V) {
        const float p = logsm ? (xr[u] - mx) - lse : expf(xr[u] - mx) / se;
        if (p > best) {
          best = p;
          bidx = c;
        }
      }
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float p = logsm ? (x[c] - mx) - lse : expf(x[c] - mx) / se;
      if (p > best) {
        best = p;
        bidx = c;
      }
    }
  }
  auto merge = [&](float ov, int oi) {
    if (ov > best || (ov == best && oi < bidx)) {
      best = ov;
      bidx = oi;
    }
  };
  merge(lane_xchg<32>(best), lane_xchg<32>(bidx));
  merge(lane_xchg<16>(best), lane_xchg<16>(bidx));
  merge(lane_xchg<8>(best), lane_xchg<8>(bidx));
  merge(lane_xchg<4>(best), lane_xchg<4>(bidx));
  merge(lane_xchg<2>(best), lane_xchg<2>(bidx));
  merge(lane_xchg<1>(best), lane_xchg<1>(bidx));
  if ((threadIdx.x & 63) == 0) {
    bv[threadIdx.x >> 6] = best;
    bi[threadIdx.x >> 6] = bidx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    best = bv[0];
    bidx = bi[0];
    for (int w = 1; w < 4; ++w)
      if (bv[w] > best || (bv[w] == best && bi[w] < bidx)) {
        best = bv[w];
        bidx = bi[w];
      }
    ids_out[(int64_t)b * ids_ld + col] = bidx;
    if (next_ids) next_ids[(int64_t)b * next_ld] = bidx;
  }
}
void argmax_softmax(const float* logits, int B, int V, int64_t* ids_out, int64_t ids_ld, int col, int32_t* next_ids,
                    int64_t next_ld, hipStream_t s, int logsm) {
  if (V <= 256 * 40) argmax_softmax_kernel<40><<<B, 256, 0, s>>>(logits, V, ids_out, ids_ld, col, next_ids, next_ld, logsm);
  else argmax_softmax_kernel<0><<<B, 256, 0, s>>>(logits, V, ids_out, ids_ld, col, next_ids, next_ld, logsm);
  CAPGEN_HIP(hipGetLastError());
}

// ---- beam search step (model.py:183-190; PolicyNetwork model_RL.py:182-190 with logsm) ----
// Candidate (j, v) of image i scores prev[j][i] + p[j*B+i][v] (p: Softmax, or LogSoftmax with
// logsm); the k best under (score desc, flat index j*V + v asc) -- a strict total order, so the
// selection equals a full sort's first k.  Part 1, one workgroup per decoder row r = j*B + i:
// the row's softmax exactly as a separate softmax pass would compute it (same strided
// per-thread order and block reductions: the scores are bit-identical), the row held in
// registers (NV values per thread; NV = 0 re-reads it from memory), each thread's sorted
// top-KM, and the row's top k.  Part 2, one wave per image: top k of its k_in rows' k
// finalists each -- every image-level winner is in its row's top k.  Neither the [R, V]
// probabilities nor a [B, k*V] scan exist: one read of the logits per step.

// sorted (desc) register top-KM insert of candidate (x, c)
template <int KM>
__device__ __forceinline__ void topk_insert(float (&tv)[KM], int (&ti)[KM], float x, int c) {
  if (!(x > tv[KM - 1] || (x == tv[KM - 1] && c < ti[KM - 1]))) return;
  float cv = x;
  int ci = c;
#pragma unroll
  for (int u = 0; u < KM; ++u) {  // unrolled: no dynamic register indexing
    const bool better = cv > tv[u] || (cv == tv[u] && ci < ti[u]);
    const float ov = tv[u];
    const int oi = ti[u];
    tv[u] = better ? cv : ov;
    ti[u] = better ? ci : oi;
    cv = better ? ov : cv;
    ci = better ? oi : ci;
  }
}

// (value, index) winner of a wave: value desc, index asc; pos rides along
template <int O>
__device__ __forceinline__ void best_step(float& best, int& bidx, int& bpos) {
  const float ov = lane_xchg<O>(best);
  const int oi = lane_xchg<O>(bidx);
  const int op = lane_xchg<O>(bpos);
  if (ov > best || (ov == best && oi < bidx)) best = ov, bidx = oi, bpos = op;
}
__device__ __forceinline__ void wave_best(float& best, int& bidx, int& bpos) {
  best_step<32>(best, bidx, bpos);
  best_step<16>(best, bidx, bpos);
  best_step<8>(best, bidx, bpos);
  best_step<4>(best, bidx, bpos);
  best_step<2>(best, bidx, bpos);
  best_step<1>(best, bidx, bpos);
}

template <int W>
__device__ __forceinline__ float blk_max(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = sh[0];
#pragma unroll
  for (int w = 1; w < W; ++w) r = fmaxf(r, sh[w]);
  __syncthreads();
  return r;
}
template <int W>
__device__ __forceinline__ float blk_sum(float v, float* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int w = 0; w < W; ++w) r += sh[w];
  __syncthreads();
  return r;
}

// NT threads per row (W = NT / 64 waves), NV values per thread in registers (V <= NT * NV)
template <int KM, int NV, int NT = 256>
__global__ void __launch_bounds__(NT) beam_row_topk_kernel(const float* __restrict__ logits,
                                                            const float* __restrict__ prev, int B, int V, int k,
                                                            int logsm, float* __restrict__ cand_v,
                                                            int* __restrict__ cand_i) {
  constexpr int W = NT / 64;
  __shared__ float sh[W];
  __shared__ float wv[W][16];
  __shared__ int wi[W][16];
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, j = r / B;
  const float* x = logits + (int64_t)r * V;
  float xr[NV > 0 ? NV : 1];
  float mx = -INFINITY;
  if constexpr (NV > 0) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int c = tid + NT * u;
      xr[u] = c < V ? x[c] : -INFINITY;
      mx = fmaxf(mx, xr[u]);
    }
  } else {
    for (int c = tid; c < V; c += NT) mx = fmaxf(mx, x[c]);
  }
  mx = blk_max<W>(mx, sh);
  float se = 0.f;
  if constexpr (NV > 0) {
#pragma unroll
    for (int u = 0; u < NV; ++u)
      if (tid + NT * u < V) {
        const float e = expf(xr[u] - mx);
        se += e;
        if (!logsm) xr[u] = e;  // Softmax scores need only exp(x - max)
      }
  } else {
    for (int c = tid; c < V; c += NT) se += expf(x[c] - mx);
  }
  se = blk_sum<W>(se, sh);
  const float lse = logf(se), add = prev ? prev[r] : 0.f;
  float tv[KM];
  int ti[KM];
#pragma unroll
  for (int u = 0; u < KM; ++u) tv[u] = -INFINITY, ti[u] = 0x7fffffff;
  if constexpr (NV > 0) {
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int c = tid + NT * u;
      if (c < V) topk_insert<KM>(tv, ti, (logsm ? (xr[u] - mx) - lse : xr[u] / se) + add, j * V + c);
    }
  } else {
    for (int c = tid; c < V; c += NT)
      topk_insert<KM>(tv, ti, (logsm ? (x[c] - mx) - lse : expf(x[c] - mx) / se) + add, j * V + c);
  }
  // the row's k best: k rounds of a wave argmax over the lanes' list heads (the winner pops its
  // head) give each wave's k best; wave 0 then selects the row's k from the 4 k of them
  for (int sel = 0; sel < k; ++sel) {
    float best = tv[0];
    int bidx = ti[0], bpos = lane;
    wave_best(best, bidx, bpos);
    if (lane == 0) wv[wave][sel] = best, wi[wave][sel] = bidx;
    if (lane == bpos) {
#pragma unroll
      for (int u = 0; u + 1 < KM; ++u) tv[u] = tv[u + 1], ti[u] = ti[u + 1];
      tv[KM - 1] = -INFINITY, ti[KM - 1] = 0x7fffffff;
    }
  }
  __syncthreads();
  if (wave == 0) {
    const bool on = lane < W * k;
    float v = on ? wv[lane / k][lane % k] : -INFINITY;
    int c = on ? wi[lane / k][lane % k] : 0x7fffffff;
    for (int sel = 0; sel < k; ++sel) {
      float best = v;
      int bidx = c, bpos = lane;
      wave_best(best, bidx, bpos);
      if (lane == 0) cand_v[(int64_t)r * k + sel] = best, cand_i[(int64_t)r * k + sel] = bidx;
      if (lane == bpos) v = -INFINITY, c = 0x7fffffff;
    }
  }
}

// one wave per image: the k best of its k_in * k row finalists (k_in * k <= 256)
__global__ void __launch_bounds__(64) beam_merge_kernel(const float* __restrict__ cand_v, const int* __restrict__ cand_i,
                                                        int k_in, int B, int V, int k, float* __restrict__ out_prob,
                                                        int32_t* __restrict__ out_src, int32_t* __restrict__ out_tok) {
  const int i = blockIdx.x, lane = threadIdx.x, n = k_in * k;
  float v[4];
  int c[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = lane + 64 * u;  // entry e = (row j = e / k, rank e % k)
    const bool on = e < n;
    const int64_t src = ((int64_t)(e / k) * B + i) * k + e % k;
    v[u] = on ? cand_v[src] : -INFINITY;
    c[u] = on ? cand_i[src] : 0x7fffffff;
  }
  for (int sel = 0; sel < k; ++sel) {
    float best = -INFINITY;
    int bidx = 0x7fffffff, bpos = -1;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (v[u] > best || (v[u] == best && c[u] < bidx)) best = v[u], bidx = c[u], bpos = lane + 64 * u;
    wave_best(best, bidx, bpos);
    if (lane == 0) {
      out_prob[sel * B + i] = best;
      out_src[sel * B + i] = bidx / V;
      out_tok[sel * B + i] = bidx % V;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (bpos == lane + 64 * u) v[u] = -INFINITY, c[u] = 0x7fffffff;
  }
}

template <int KM>
static void beam_row_topk(const float* logits, const float* prev, int rows, int B, int V, int k, int logsm,
                          float* cand_v, int32_t* cand_i, hipStream_t s) {
  // 512 threads per row where the row fits 20 values per thread (42 vs 50 us per token at B = 1280
  // with 256 threads, round 2)
  if (V <= 512 * 20 && KM * 8 <= 64)
    beam_row_topk_kernel<KM, 20, 512><<<rows, 512, 0, s>>>(logits, prev, B, V, k, logsm, cand_v, cand_i);
  else if (V <= 256 * 40) beam_row_topk_kernel<KM, 40><<<rows, 256, 0, s>>>(logits, prev, B, V, k, logsm, cand_v, cand_i);
  else beam_row_topk_kernel<KM, 0><<<rows, 256, 0, s>>>(logits, prev, B, V, k, logsm, cand_v, cand_i);
}

void beam_step_topk(const float* logits, const float* prev, int k_in, int B, int V, int k, int logsm, float* cand_v,
                    int32_t* cand_i, float* out_prob, int32_t* out_src, int32_t* out_tok, hipStream_t s) {
  require(k >= 1 && k <= 16 && k_in >= 1 && k_in * k <= 256, "beam_step_topk: k in [1, 16]");
  const int rows = k_in * B;
  if (k <= 4) beam_row_topk<4>(logits, prev, rows, B, V, k, logsm, cand_v, cand_i, s);
  else if (k == 5) beam_row_topk<5>(logits, prev, rows, B, V, k, logsm, cand_v, cand_i, s);
  else if (k <= 8) beam_row_topk<8>(logits, prev, rows, B, V, k, logsm, cand_v, cand_i, s);
  else beam_row_topk<16>(logits, prev, rows, B, V, k, logsm, cand_v, cand_i, s);
  beam_merge_kernel<<<B, 64, 0, s>>>(cand_v, cand_i, k_in, B, V, k, out_prob, out_src, out_tok);
  CAPGEN_HIP(hipGetLastError());
}

// ---- bf16 decode selection from slab stats (GemmArgs::dec_stats) ----------------------------
// One wave per row, 4 rows per workgroup.  The row's ceil(V/16) slab stats (8 B each, 1/8 of the
// f32 logits) sit NS per lane in registers: one pass gives the row max M and the exp-sum
// se = sum_c s_c exp(m_c - M) (the softmax of the selected elements is exp(x - M) / se), and each
// lane's sorted best slabs.  Any element of the row's top k (value desc, index asc) lies in one of
// the k best slabs under (max desc, slab asc): every slab ranked before the slab of the k-th best
// element holds, as its maximum, a distinct element ranked before it.  So only k * 16 logits are
// read back.  (The softmax is monotone in the logit; two logits rounding to one probability could
// order by index differently than a full scan would -- the bf16 path is held to the fp32 engine by
// the top-2-margin tests, the fp32 parity path keeps the exact full-row kernels above.)
constexpr int kSlabNS = 16;  // slabs per lane: V <= 64 * 16 * 16 = 16384
bool slab_select_ok(int V) { return V >= 1 && (V + 15) / 16 <= 64 * kSlabNS; }

struct SlabRow {
  float M, se;
};
// the row max and exp-sum from the stats; every lane ends with both
__device__ __forceinline__ SlabRow slab_row_stats(const float2* __restrict__ st, int S, int lane, float (&mx)[kSlabNS]) {
  float2 x[kSlabNS];
  float M = -INFINITY;
#pragma unroll
  for (int u = 0; u < kSlabNS; ++u) {
    const int c = lane + 64 * u;
    x[u] = c < S ? st[c] : float2{-INFINITY, 0.f};
    mx[u] = x[u].x;
    M = fmaxf(M, x[u].x);
  }
  M = wave_max(M);
  float se = 0.f;
#pragma unroll
  for (int u = 0; u < kSlabNS; ++u)
    if (lane + 64 * u < S) se += x[u].y * __expf(x[u].x - M);
  return SlabRow{M, wave_sum(se)};
}

__global__ void __launch_bounds__(256) slab_argmax_kernel(const float* __restrict__ logits,
                                                          const float2* __restrict__ stats, int B, int V,
                                                          int64_t* __restrict__ ids_out, int64_t ids_ld, int col,
                                                          int32_t* __restrict__ next_ids, int64_t next_ld) {
  const int lane = threadIdx.x & 63, b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // (whole waves)
  const int S = (V + 15) / 16;
  const float2* st = stats + (int64_t)b * S;
  // best slab of this lane (max desc, slab asc), then of the wave
  float best = -INFINITY;
  int bidx = 0x7fffffff, bpos = lane;
#pragma unroll
  for (int u = 0; u < kSlabNS; ++u) {
    const int c = lane + 64 * u;
    if (c < S) {
      const float m = st[c].x;
      if (m > best) best = m, bidx = c;  // c ascends: ties keep the first
    }
  }
  wave_best(best, bidx, bpos);
  // the slab's 16 logits: the first column holding the maximum
  const int c = bidx * 16 + lane;
  float v = -INFINITY;
  int vi = 0x7fffffff, vp = lane;
  if (lane < 16 && c < V) v = logits[(int64_t)b * V + c], vi = c;
  wave_best(v, vi, vp);
  if (lane == 0) {
    ids_out[(int64_t)b * ids_ld + col] = vi;
    if (next_ids) next_ids[(int64_t)b * next_ld] = vi;
  }
}
void slab_argmax(const float* logits, const float2* stats, int B, int V, int64_t* ids_out, int64_t ids_ld, int col,
                 int32_t* next_ids, int64_t next_ld, hipStream_t s) {
  require(slab_select_ok(V), "slab_argmax: V must be in [1, 16384]");
  slab_argmax_kernel<<<(B + 3) / 4, 256, 0, s>>>(logits, stats, B, V, ids_out, ids_ld, col, next_ids, next_ld);
  CAPGEN_HIP(hipGetLastError());
}

// one row's k best (value desc, index asc) from its slab stats: a wave per row, lane 0 leaves them in
// (out_v, out_i)[0 .. k); chosen = this wave's KM-entry LDS scratch (row j = beam index)
template <int KM>
__device__ __forceinline__ void slab_row_topk_wave(const float* __restrict__ logits, const float2* __restrict__ stats,
                                                   const float* __restrict__ prev, int r, int j, int V, int k,
                                                   int logsm, int* chosen, int lane, float* out_v, int* out_i) {
  const int S = (V + 15) / 16;
  float mx[kSlabNS];
  const SlabRow rs = slab_row_stats(stats + (int64_t)r * S, S, lane, mx);
  // each lane's best KM slabs, sorted; then k wave rounds pick the row's k best slabs
  float tv[KM];
  int ti[KM];
#pragma unroll
  for (int u = 0; u < KM; ++u) tv[u] = -INFINITY, ti[u] = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < kSlabNS; ++u) {
    const int c = lane + 64 * u;
    if (c < S) topk_insert<KM>(tv, ti, mx[u], c);
  }
  for (int sel = 0; sel < k; ++sel) {
    float best = tv[0];
    int bidx = ti[0], bpos = lane;
    wave_best(best, bidx, bpos);
    if (lane == 0) chosen[sel] = bidx;  // (0x7fffffff when S < k: no such slab)
    if (lane == bpos) {
#pragma unroll
      for (int u = 0; u + 1 < KM; ++u) tv[u] = tv[u + 1], ti[u] = ti[u + 1];
      tv[KM - 1] = -INFINITY, ti[KM - 1] = 0x7fffffff;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // lane 0's LDS writes before the reads below
  // the k * 16 candidate logits, scored exactly as the full-row kernel scores them
  const float lse = __logf(rs.se), add = prev ? prev[r] : 0.f;
#pragma unroll
  for (int u = 0; u < KM; ++u) tv[u] = -INFINITY, ti[u] = 0x7fffffff;
  const float* x = logits + (int64_t)r * V;
  for (int e = lane; e < k * 16; e += 64) {
    const int sl = chosen[e >> 4];
    if (sl == 0x7fffffff) continue;
    const int c = sl * 16 + (e & 15);
    if (c >= V) continue;
    const float xv = x[c];
    topk_insert<KM>(tv, ti, (logsm ? (xv - rs.M) - lse : __expf(xv - rs.M) / rs.se) + add, j * V + c);
  }
  for (int sel = 0; sel < k; ++sel) {
    float best = tv[0];
    int bidx = ti[0], bpos = lane;
    wave_best(best, bidx, bpos);
    if (lane == 0) out_v[sel] = best, out_i[sel] = bidx;
    if (lane == bpos) {
#pragma unroll
      for (int u = 0; u + 1 < KM; ++u) tv[u] = tv[u + 1], ti[u] = ti[u + 1];
      tv[KM - 1] = -INFINITY, ti[KM - 1] = 0x7fffffff;
    }
  }
}

template <int KM>
__global__ void __launch_bounds__(256) slab_row_topk_kernel(const float* __restrict__ logits,
                                                            const float2* __restrict__ stats,
                                                            const float* __restrict__ prev, int rows, int B, int V,
                                                            int k, int logsm, float* __restrict__ cand_v,
                                                            int* __restrict__ cand_i) {
  __shared__ int chosen[4][KM];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = blockIdx.x * 4 + wave;
  if (r >= rows) return;  // (whole waves; no workgroup barrier below)
  slab_row_topk_wave<KM>(logits, stats, prev, r, r / B, V, k, logsm, chosen[wave], lane, cand_v + (int64_t)r * k,
                         cand_i + (int64_t)r * k);
}

// The whole beam step of one image in ONE workgroup (round 6): wave j takes beam row j * B + i's k best
// (slab_row_topk_wave) into LDS, wave 0 merges the k_in * k finalists exactly as beam_merge_kernel, and
// every thread then moves the image's k new rows -- sequences and ids gathered from their source beams
// with the chosen token at column t + 1, and the beam K/V row table (model.py:186-198) -- which took
// four more launches (merge, two gathers, the row table) per token.
template <int KM>
__global__ void __launch_bounds__(1024) beam_slab_step_kernel(
    const float* __restrict__ logits, const float2* __restrict__ stats, const float* __restrict__ prev, int k_in,
    int B, int V, int k, int logsm, float* __restrict__ out_prob, int32_t* __restrict__ out_src,
    int32_t* __restrict__ out_tok, const int64_t* __restrict__ seq_src, int64_t* __restrict__ seq_dst, int Tw,
    const int32_t* __restrict__ ids_src, int32_t* __restrict__ ids_dst, const int32_t* __restrict__ kv_src,
    int32_t* __restrict__ kv_dst, int Tc, int t) {
  __shared__ int chosen[16][KM];
  __shared__ float cv[256];
  __shared__ int ci[256];
  __shared__ int bsrc[16], btok[16];
  const int i = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave < k_in)
    slab_row_topk_wave<KM>(logits, stats, prev, wave * B + i, wave, V, k, logsm, chosen[wave], lane, cv + wave * k,
                           ci + wave * k);
  __syncthreads();
  if (wave == 0) {  // beam_merge_kernel over the LDS finalists (entry e = row e / k, rank e % k)
    const int n = k_in * k;
    float v[4];
    int c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = lane + 64 * u;
      const bool on = e < n;
      v[u] = on ? cv[e] : -INFINITY;
      c[u] = on ? ci[e] : 0x7fffffff;
    }
    for (int sel = 0; sel < k; ++sel) {
      float best = -INFINITY;
      int bidx = 0x7fffffff, bpos = -1;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (v[u] > best || (v[u] == best && c[u] < bidx)) best = v[u], bidx = c[u], bpos = lane + 64 * u;
      wave_best(best, bidx, bpos);
      if (lane == 0) {
        out_prob[sel * B + i] = best;
        out_src[sel * B + i] = bsrc[sel] = bidx / V;
        out_tok[sel * B + i] = btok[sel] = bidx % V;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (bpos == lane + 64 * u) v[u] = -INFINITY, c[u] = 0x7fffffff;
    }
  }
  __syncthreads();
  // the image's k new rows r = j * B + i from their source rows bsrc[j] * B + i (double-buffered arrays)
  for (int e = threadIdx.x; e < k * (Tw + 2 * Tc); e += blockDim.x) {
    const int j = e / (Tw + 2 * Tc), q = e % (Tw + 2 * Tc);
    const int64_t r = (int64_t)j * B + i, srow = (int64_t)bsrc[j] * B + i;
    if (q < Tw) {
      seq_dst[r * Tw + q] = q == t + 1 ? (int64_t)btok[j] : seq_src[srow * Tw + q];
    } else if (q < Tw + Tc) {
      const int cc = q - Tw;
      ids_dst[r * Tc + cc] = cc == t + 1 ? btok[j] : ids_src[srow * Tc + cc];
    } else {
      const int cc = q - Tw - Tc;
      kv_dst[r * Tc + cc] = cc <= t ? kv_src[srow * Tc + cc] : (cc == t + 1 ? (int32_t)r : 0);
    }
  }
}

void beam_slab_step(const float* logits, const float2* stats, const float* prev, int k_in, int B, int V, int k,
                    int logsm, float* out_prob, int32_t* out_src, int32_t* out_tok, const int64_t* seq_src,
                    int64_t* seq_dst, int Tw, const int32_t* ids_src, int32_t* ids_dst, const int32_t* kv_src,
                    int32_t* kv_dst, int Tc, int t, hipStream_t s) {
  require(k >= 1 && k <= 16 && k_in >= 1 && k_in <= 16 && k_in * k <= 256, "beam_slab_step: k, k_in in [1, 16]");
  require(slab_select_ok(V) && t + 1 < Tw && t + 1 < Tc, "beam_slab_step: V in [1, 16384], t + 1 < width");
  if (hz::active()) {
    using namespace hz;
    const int R = k * B, S = (V + 15) / 16;
    op(s, "beam_slab_step", {rd(logits, (int64_t)k_in * B * V * 4), rd(stats, (int64_t)k_in * B * S * 8),
                             rd(prev, prev ? (int64_t)k_in * B * 4 : 0), wr(out_prob, (int64_t)k * B * 4),
                             wr(out_src, (int64_t)k * B * 4), wr(out_tok, (int64_t)k * B * 4),
                             rd(seq_src, (int64_t)R * Tw * 8), wr(seq_dst, (int64_t)R * Tw * 8),
                             rd(ids_src, (int64_t)R * Tc * 4), wr(ids_dst, (int64_t)R * Tc * 4),
                             rd(kv_src, (int64_t)R * Tc * 4), wr(kv_dst, (int64_t)R * Tc * 4)});
  }
  const int nt = 64 * k_in;
  auto go = [&](auto km) {
    beam_slab_step_kernel<decltype(km)::value><<<B, nt, 0, s>>>(logits, stats, prev, k_in, B, V, k, logsm, out_prob,
                                                                out_src, out_tok, seq_src, seq_dst, Tw, ids_src,
                                                                ids_dst, kv_src, kv_dst, Tc, t);
  };
  if (k <= 4) go(std::integral_constant<int, 4>{});
  else if (k == 5) go(std::integral_constant<int, 5>{});
  else if (k <= 8) go(std::integral_constant<int, 8>{});
  else go(std::integral_constant<int, 16>{});
  CAPGEN_HIP(hipGetLastError());
}

void beam_step_topk_slab(const float* logits, const float2* stats, const float* prev, int k_in, int B, int V, int k,
                         int logsm, float* cand_v, int32_t* cand_i, float* out_prob, int32_t* out_src,
                         int32_t* out_tok, hipStream_t s) {
  require(k >= 1 && k <= 16 && k_in >= 1 && k_in * k <= 256, "beam_step_topk_slab: k in [1, 16]");
  require(slab_select_ok(V), "beam_step_topk_slab: V must be in [1, 16384]");
  const int rows = k_in * B, grid = (rows + 3) / 4;
  if (k <= 4) slab_row_topk_kernel<4><<<grid, 256, 0, s>>>(logits, stats, prev, rows, B, V, k, logsm, cand_v, cand_i);
  else if (k == 5) slab_row_topk_kernel<5><<<grid, 256, 0, s>>>(logits, stats, prev, rows, B, V, k, logsm, cand_v, cand_i);
  else if (k <= 8) slab_row_topk_kernel<8><<<grid, 256, 0, s>>>(logits, stats, prev, rows, B, V, k, logsm, cand_v, cand_i);
  else slab_row_topk_kernel<16><<<grid, 256, 0, s>>>(logits, stats, prev, rows, B, V, k, logsm, cand_v, cand_i);
  beam_merge_kernel<<<B, 64, 0, s>>>(cand_v, cand_i, k_in, B, V, k, out_prob, out_src, out_tok);
  CAPGEN_HIP(hipGetLastError());
}

__global__ void bump_seed_kernel(uint64_t* seed) { *seed += 0x9E3779B97F4A7C15ull; }
void bump_seed(uint64_t* seed, hipStream_t s) {
  bump_seed_kernel<<<1, 1, 0, s>>>(seed);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
