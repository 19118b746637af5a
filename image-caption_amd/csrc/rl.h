// capgen — SCST (self-critical) loss kernels, see rl.hip.
#pragma once
#include "capgen_common.h"
#include "gemm.h"

namespace capgen {

// per logit row: sample (argmax log_softmax), log-sum-exp, logp[sample], entropy
void rl_rows(const float* logits, int M, int V, int32_t* sample, float* lse, float* logp_s, float* ent,
             hipStream_t s);
// per image masked mean entropy (B), scal[0] = local sum(mask)
void rl_image(const int32_t* sample, const float* ent, int B, int L, float* ent_img, float* scal, hipStream_t s);
// scal[1] = local -sum logp[sample] * mask * score_b
void rl_numer(const int32_t* sample, const float* logp_s, const float* score, int B, int L, float* scal,
              hipStream_t s);
// out = {(1-w) lm + w struct, lm, struct}, struct = scal[1] / scal[0]; grad_scale = 1
void rl_loss(const float* scal, const float* lm, float w, float* out, float* grad_scale, hipStream_t s);
// fully scaled d(loss)/d(logits) for the combined LM + structure loss
void rl_grad(const float* logits, const int32_t* tgt, const int32_t* sample, const float* lse, const float* score,
             const float* count, const float* scal, int B, int L, int V, int pad, float w, void* dl, DType t,
             hipStream_t s);
void rl_export(const int32_t* sample, int n, int64_t* out, hipStream_t s);

}  // namespace capgen
