// capgen — bf16 MFMA attention for short sequences (Lq, Lk <= 64, head size 64), one
// workgroup of four wave64s per (batch, head).  Used by the bf16 performance path; the f32
// parity path keeps the exact-order VALU kernels of attention.hip.
//
// Every product is a v_mfma_f32_16x16x32_bf16 issued with swapped operands, so a lane ends
// with 4 CONSECUTIVE columns of one row: lane l holds X[row = l&15][col = 16t + 4(l>>4) + r].
// That register layout is exactly the permuted-K operand order of gemm_bf16.hip (lane group
// g carries k = 4g..4g+3 and 16+4g..16+4g+3 of each 32-deep step), so the softmax output P and
// the score gradient dS feed the next MFMA straight from registers, with no LDS round trip.
// Operands whose K dimension runs down memory rows (V^T, K^T, dO^T, Q^T, Pd^T, dS^T) are read
// from [64][64] bf16 LDS images with ds_read_b64_tr_b16, XOR-swizzled per row.
//
// Forward  (wave w = query rows 16w..16w+15):  S = (Q K^T)/temperature -> mask -> softmax
//          (row max/sum: 16 values in registers + 2 cross-lane steps) -> [probs] -> dropout
//          -> O = P V.
// Backward (recomputes P; probs are not read):  dPd = dO V^T, dropout, dS = P (dP - rowsum),
//          dQ = dS K / temperature (wave = query tile), then through LDS images of Pd and dS:
//          dV = Pd^T dO, dK = dS^T Q / temperature (wave = key tile).
// Semantics as attention.hip (modules.py:16-27): same masks, same counter-based dropout index.
#include <cstdlib>

#include "attention.h"
#include "attn_mfma_dev.h"

namespace capgen {
using namespace amf;

__global__ void __launch_bounds__(256) attn_fwd_mfma_kernel(AttnGeom g, bf16* __restrict__ o,
                                                            float* __restrict__ probs) {
  __shared__ __attribute__((aligned(16))) char sm[kFwdSmem];
  StampScope stamp_scope(g.stamp);
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  attn_fwd_one(g, o, probs, blockIdx.x / g.H, blockIdx.x % g.H, sm);
}

// One wave64 per (batch, head) when every query row fits one 16-row tile (Lq <= 16: the beam's
// cross attention at decode, an image's k beam rows over its keys).  The Q image holds only those
// 16 rows: 2 + 8 + 8 KB + the key flags = 18.1 KB of LDS, so eight workgroups share a CU and the
// decode's B * H = 2048 (image, head) pairs run in one round; the 4-wave kernel holds 24.6 KB
// (six per CU, two rounds) and leaves three of its waves idle at Lq <= 16.  Same arithmetic as the
// 4-wave kernel's wave 0 (attn_fwd_images): bit-identical results.
__global__ void __launch_bounds__(64) attn_fwd_wave_kernel(AttnGeom g, bf16* __restrict__ o,
                                                           float* __restrict__ probs) {
  __shared__ __attribute__((aligned(16))) char sm[2 * IMG + 16 * 128 + 64];
  StampScope stamp_scope(g.stamp);
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  char* Kimg = sm;
  char* Vimg = sm + IMG;
  char* Qimg = sm + 2 * IMG;
  unsigned char* kok = reinterpret_cast<unsigned char*>(sm + 2 * IMG + 16 * 128);
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H, lane = threadIdx.x;
  const int bk = g.kv_bmod ? b % g.kv_bmod : b;
  const bf16* kb = reinterpret_cast<const bf16*>(g.k) + (int64_t)bk * g.k_bs + h * DK;
  const bf16* vb = reinterpret_cast<const bf16*>(g.v) + (int64_t)bk * g.v_bs + h * DK;
  const bf16* qb = reinterpret_cast<const bf16*>(g.q) + (int64_t)b * g.q_bs + h * DK;
  // every load first (K / V: 64 rows x 8 chunks of 16 B, rows >= Lk zero; Q: 16 rows).  The loads
  // of rows past Lk are skipped, not clamped: the kernel is bound by its load issue (clamped
  // redundant loads of the last row measured 20.6 vs 9.4 us per launch at C4)
  uint4 kv[2][8], qv[2];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = lane + 64 * u, row = c >> 3, ch = c & 7;
    kv[0][u] = row < g.Lk ? *reinterpret_cast<const uint4*>(kb + (int64_t)row * g.k_ld + ch * 8) : uint4{0u, 0u, 0u, 0u};
    kv[1][u] = row < g.Lk ? *reinterpret_cast<const uint4*>(vb + (int64_t)row * g.v_ld + ch * 8) : uint4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = lane + 64 * u, row = c >> 3, ch = c & 7;
    qv[u] = row < g.Lq ? *reinterpret_cast<const uint4*>(qb + (int64_t)row * g.q_ld + ch * 8) : uint4{0u, 0u, 0u, 0u};
  }
  stage_key_ok(kok, g, b, lane);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int c = lane + 64 * u, row = c >> 3, ch = c & 7;
    *reinterpret_cast<uint4*>(Kimg + row * 128 + swz(row, ch) * 16) = kv[0][u];
    *reinterpret_cast<uint4*>(Vimg + row * 128 + swz(row, ch) * 16) = kv[1][u];
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = lane + 64 * u, row = c >> 3, ch = c & 7;
    *reinterpret_cast<uint4*>(Qimg + row * 128 + swz(row, ch) * 16) = qv[u];
  }
  __syncthreads();
  attn_fwd_images(g, o, probs, b, h, Qimg, Kimg, Vimg, kok);
}

__global__ void __launch_bounds__(256) attn_bwd_mfma_kernel(AttnGeom g, const bf16* __restrict__ dout,
                                                            bf16* __restrict__ dq, bf16* __restrict__ dkp,
                                                            bf16* __restrict__ dvp) {
  __shared__ __attribute__((aligned(16))) char sm[6 * IMG + 64];
  StampScope stamp_scope(g.stamp);
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  char* Kimg = sm;             // [key][d]
  char* dOimg = sm + IMG;      // [q][d]
  char* Qimg = sm + 2 * IMG;   // [q][d]
  char* Vimg = sm + 3 * IMG;   // [key][d]
  char* Pdimg = sm + 4 * IMG;  // [q][key]  dropped probabilities
  char* dSimg = sm + 5 * IMG;  // [q][key]  score gradient
  unsigned char* kok = reinterpret_cast<unsigned char*>(sm + 6 * IMG);
  const int b = blockIdx.x / g.H, h = blockIdx.x % g.H;
  const int tid = threadIdx.x;
  const int64_t qoff = (int64_t)b * g.q_bs + h * DK, koff = (int64_t)b * g.k_bs + h * DK,
                voff = (int64_t)b * g.v_bs + h * DK, ooff = (int64_t)b * g.o_bs + h * DK;
  const bf16* qb = reinterpret_cast<const bf16*>(g.q) + qoff;
  const bf16* kb = reinterpret_cast<const bf16*>(g.k) + koff;
  const bf16* vb = reinterpret_cast<const bf16*>(g.v) + voff;
  const bf16* dob = dout + ooff;
  {
    char* const img[4] = {Kimg, dOimg, Qimg, Vimg};
    const bf16* const src[4] = {kb, dob, qb, vb};
    const int64_t ld[4] = {g.k_ld, g.o_ld, g.q_ld, g.v_ld};
    const int L[4] = {g.Lk, g.Lq, g.Lq, g.Lk};
    stage_images<4>(img, src, ld, L, tid);
    stage_key_ok(kok, g, b, tid);
  }
  __syncthreads();

  attn_bwd_staged(g, dq, dkp, dvp, b, h, Kimg, dOimg, Qimg, Vimg, Pdimg, dSimg, kok);
}

bool attention_mfma_ok(const AttnGeom& g) {
  return g.dk == DK && g.Lq <= 64 && g.Lk <= 64 && g.q_ld % 8 == 0 && g.k_ld % 8 == 0 && g.v_ld % 8 == 0 &&
         g.o_ld % 8 == 0 && g.q_bs % 8 == 0 && g.k_bs % 8 == 0 && g.v_bs % 8 == 0 && g.o_bs % 8 == 0;
}

void attention_fwd_mfma(const AttnGeom& g, bf16* o, float* probs, hipStream_t s) {
  // Knob::AttnWave = 0: the 4-wave kernel (bit-identity test)
  if (g.Lq <= 16) {
    if (knob(Knob::AttnWave)) {
      attn_fwd_wave_kernel<<<g.B * g.H, 64, 0, s>>>(g, o, probs);
      CAPGEN_HIP(hipGetLastError());
      return;
    }
  }
  attn_fwd_mfma_kernel<<<g.B * g.H, 256, 0, s>>>(g, o, probs);
  CAPGEN_HIP(hipGetLastError());
}

void attention_bwd_mfma(const AttnGeom& g, const bf16* dout, bf16* dq, bf16* dk, bf16* dv, hipStream_t s) {
  attn_bwd_mfma_kernel<<<g.B * g.H, 256, 0, s>>>(g, dout, dq, dk, dv);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
