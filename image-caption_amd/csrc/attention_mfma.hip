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
  static const bool off = std::getenv("CAPGEN_ATTN_VALU") != nullptr;  // A/B experiment knob
  return !off && g.dk == DK && g.Lq <= 64 && g.Lk <= 64 && g.q_ld % 8 == 0 && g.k_ld % 8 == 0 && g.v_ld % 8 == 0 &&
         g.o_ld % 8 == 0 && g.q_bs % 8 == 0 && g.k_bs % 8 == 0 && g.v_bs % 8 == 0 && g.o_bs % 8 == 0;
}

void attention_fwd_mfma(const AttnGeom& g, bf16* o, float* probs, hipStream_t s) {
  attn_fwd_mfma_kernel<<<g.B * g.H, 256, 0, s>>>(g, o, probs);
  CAPGEN_HIP(hipGetLastError());
}

void attention_bwd_mfma(const AttnGeom& g, const bf16* dout, bf16* dq, bf16* dk, bf16* dv, hipStream_t s) {
  attn_bwd_mfma_kernel<<<g.B * g.H, 256, 0, s>>>(g, dout, dq, dk, dv);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
