// capgen — masked multi-head attention (forward/backward) launcher interface.
#pragma once
#include "capgen_common.h"
#include "gemm.h"

namespace capgen {

// Row (b, i) of head h of a [.., H*dk] activation lives at base + b*bs + i*ld + h*dk.
struct AttnGeom {
  int B = 0, H = 0, Lq = 0, Lk = 0, dk = 0;
  int prio = 0;  // 1: raise the waves' issue priority (critical path)
  const void* q = nullptr; int64_t q_ld = 0, q_bs = 0;
  const void* k = nullptr; int64_t k_ld = 0, k_bs = 0;
  const void* v = nullptr; int64_t v_ld = 0, v_bs = 0;
  int kv_bmod = 0;                    // > 0: K/V/key_valid of query batch b come from batch b % kv_bmod
  // decode only (Lq = 1): key j of query batch b is stored in batch kv_row[b*kv_row_ld + j]
  // (beam search: a beam's cached K/V positions live in the rows of the beams it descends from)
  const int32_t* kv_row = nullptr; int64_t kv_row_ld = 0;
  int64_t o_ld = 0, o_bs = 0;         // layout of O (forward output) and dO (backward input)
  // key mask: key (b, j) is masked if key_valid[b*kv_bs + j] == 0, or key_ids[b*kid_bs + j] == pad
  const uint8_t* key_valid = nullptr; int64_t kv_bs = 0;
  const int32_t* key_ids = nullptr; int64_t kid_bs = 0; int pad_idx = 0;
  int causal = 0, q_pos0 = 0;         // mask keys j > q_pos0 + i
  float temperature = 1.f;            // sqrt(dk), q is divided by it (modules.py:18,56)
  Drop drop{};                        // dropout on the probabilities (modules.py:24)
  uint64_t* stamp = nullptr;          // diagnostic timestamps (StampScope)
};

// probs (optional): [B,H,Lq,Lk] f32, pre-dropout softmax, saved for backward / attention_list.
void attention_fwd(const AttnGeom& g, void* o, float* probs, DType t, hipStream_t s);
// dq/dk/dv mirror the q/k/v layouts (same ld/bs).  dO uses o_ld/o_bs.
void attention_bwd(const AttnGeom& g, const float* probs, const void* dout, void* dq, void* dk,
                   void* dv, DType t, hipStream_t s);
// bf16 MFMA kernels (attention_mfma.hip), used by attention_fwd/bwd when attention_mfma_ok(g);
// the backward recomputes the probabilities and never reads `probs`
bool attention_mfma_ok(const AttnGeom& g);
void attention_fwd_mfma(const AttnGeom& g, bf16* o, float* probs, hipStream_t s);
void attention_bwd_mfma(const AttnGeom& g, const bf16* dout, bf16* dq, bf16* dk, bf16* dv, hipStream_t s);
// out[b*N + j] = mean over heads of probs[b, :, row, j]   (model.py:123)
void attention_head_mean(const float* probs, int B, int H, int Lq, int Lk, int row, float* out,
                         hipStream_t s);

}  // namespace capgen
