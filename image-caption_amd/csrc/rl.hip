// capgen — self-critical sequence training (SCST) kernels: the device side of
// SelfCriticNetwork.train_step (models.py:179-195), PolicyNetwork.sample (model_RL.py:93-97)
// and ReinforcementLearningLoss / StructureCriterion (loss.py:53-76, 115-152).  The CIDEr-D /
// BLEU rewards are computed on the host between rl_sample and rl_finish (capgen/scst.py).
//
//   rows  : per logit row m = (b, t): lse, sample = argmax(log_softmax) (first index on ties),
//           logp[sample], entropy = -sum p log p                           (model_RL.py:93-97)
//   image : mask_bt = 1 (t = 0) or sample[b, t-1] > 0; per-image masked mean entropy; sum(mask)
//   loss  : struct = -sum logp[sample] * mask * score_b / sum(mask);  loss = (1-w) lm + w struct
//   grad  : dlogits = a (softmax - onehot(tgt)) + c (softmax - onehot(sample)),
//           a = (1-w)/count [tgt != pad], c = w score_b mask_bt / sum(mask)
// All-reduced scalars (DP): count (forward), sum(mask) and the struct numerator (rl_finish).
#include "rl.h"

namespace capgen {

namespace {
__device__ __forceinline__ float bmax(float v, float* sh) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ float bsum(float v, float* sh) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();
  return r;
}
}  // namespace

__global__ void __launch_bounds__(256) rl_rows_kernel(const float* __restrict__ logits, int V,
                                                      int32_t* __restrict__ sample, float* __restrict__ lse,
                                                      float* __restrict__ logp_s, float* __restrict__ ent) {
  __shared__ float sh[4];
  __shared__ float bv[4];
  __shared__ int bi[4];
  const int m = blockIdx.x;
  const float* x = logits + (int64_t)m * V;
  float mx = -INFINITY;
  for (int c = threadIdx.x; c < V; c += 256) mx = fmaxf(mx, x[c]);
  mx = bmax(mx, sh);
  float se = 0.f, sx = 0.f;
  for (int c = threadIdx.x; c < V; c += 256) {
    const float e = expf(x[c] - mx);
    se += e;
    sx = fmaf(e, x[c] - mx, sx);
  }
  se = bsum(se, sh);
  sx = bsum(sx, sh);
  const float lz = logf(se);
  // argmax of log_softmax = (x - max) - log(sum), first index on ties (torch.argmax)
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int c = threadIdx.x; c < V; c += 256) {
    const float lp = (x[c] - mx) - lz;
    if (lp > best) best = lp, bidx = c;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ov > best || (ov == best && oi < bidx)) best = ov, bidx = oi;
  }
  if ((threadIdx.x & 63) == 0) bv[threadIdx.x >> 6] = best, bi[threadIdx.x >> 6] = bidx;
  __syncthreads();
  if (threadIdx.x == 0) {
    best = bv[0], bidx = bi[0];
    for (int w = 1; w < 4; ++w)
      if (bv[w] > best || (bv[w] == best && bi[w] < bidx)) best = bv[w], bidx = bi[w];
    sample[m] = bidx;
    lse[m] = mx + lz;
    logp_s[m] = best;
    ent[m] = lz - sx / se;  // -sum p (x - max - lz)
  }
}

// one workgroup: per-image masked entropy mean, local sum(mask) -> scal[0]
__global__ void __launch_bounds__(256) rl_image_kernel(const int32_t* __restrict__ sample,
                                                       const float* __restrict__ ent, int B, int L,
                                                       float* __restrict__ ent_img, float* __restrict__ scal) {
  __shared__ float sh[4];
  float msum = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    float es = 0.f, ms = 0.f;
    for (int t = 0; t < L; ++t) {
      const float mk = (t == 0 || sample[b * L + t - 1] > 0) ? 1.f : 0.f;
      es = fmaf(ent[b * L + t], mk, es);
      ms += mk;
    }
    ent_img[b] = es / ms;
    msum += ms;
  }
  msum = bsum(msum, sh);
  if (threadIdx.x == 0) scal[0] = msum;
}

// local struct numerator -sum logp * mask * score -> scal[1]
__global__ void __launch_bounds__(256) rl_numer_kernel(const int32_t* __restrict__ sample,
                                                       const float* __restrict__ logp_s,
                                                       const float* __restrict__ score, int B, int L,
                                                       float* __restrict__ scal) {
  __shared__ float sh[4];
  float acc = 0.f;
  for (int m = threadIdx.x; m < B * L; m += 256) {
    const int b = m / L, t = m % L;
    const float mk = (t == 0 || sample[m - 1] > 0) ? 1.f : 0.f;
    acc = fmaf(-logp_s[m] * mk, score[b], acc);
  }
  acc = bsum(acc, sh);
  if (threadIdx.x == 0) scal[1] = acc;
}

__global__ void rl_loss_kernel(const float* __restrict__ scal, const float* __restrict__ lm, float w,
                               float* __restrict__ out, float* __restrict__ grad_scale) {
  const float st = scal[1] / scal[0];
  const float l = w < 1.f ? *lm : 0.f;
  out[0] = (1.f - w) * l + w * st;
  out[1] = l;
  out[2] = st;
  *grad_scale = 1.f;  // rl_grad writes fully scaled dlogits
}

template <typename T>
__global__ void __launch_bounds__(256) rl_grad_kernel(const float* __restrict__ logits, const int32_t* __restrict__ tgt,
                                                      const int32_t* __restrict__ sample, const float* __restrict__ lse,
                                                      const float* __restrict__ score, const float* __restrict__ count,
                                                      const float* __restrict__ scal, int L, int V, int pad, float w,
                                                      T* __restrict__ dl) {
  const int m = blockIdx.x, b = m / L, t = m % L;
  const float* x = logits + (int64_t)m * V;
  T* g = dl + (int64_t)m * V;
  const int y = tgt[m], sm = sample[m];
  const float mk = (t == 0 || sample[m - 1] > 0) ? 1.f : 0.f;
  const float a = (y != pad && w < 1.f) ? (1.f - w) / *count : 0.f;
  const float c = w * score[b] * mk / scal[0];
  const float z = lse[m];
  for (int v = threadIdx.x; v < V; v += 256) {
    const float p = expf(x[v] - z);
    g[v] = from_f<T>((a + c) * p - (v == y ? a : 0.f) - (v == sm ? c : 0.f));
  }
}

__global__ void rl_export_kernel(const int32_t* __restrict__ sample, int n, int64_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = sample[i];
}

void rl_rows(const float* logits, int M, int V, int32_t* sample, float* lse, float* logp_s, float* ent,
             hipStream_t s) {
  rl_rows_kernel<<<M, 256, 0, s>>>(logits, V, sample, lse, logp_s, ent);
  CAPGEN_HIP(hipGetLastError());
}
void rl_image(const int32_t* sample, const float* ent, int B, int L, float* ent_img, float* scal, hipStream_t s) {
  rl_image_kernel<<<1, 256, 0, s>>>(sample, ent, B, L, ent_img, scal);
  CAPGEN_HIP(hipGetLastError());
}
void rl_numer(const int32_t* sample, const float* logp_s, const float* score, int B, int L, float* scal,
              hipStream_t s) {
  rl_numer_kernel<<<1, 256, 0, s>>>(sample, logp_s, score, B, L, scal);
  CAPGEN_HIP(hipGetLastError());
}
void rl_loss(const float* scal, const float* lm, float w, float* out, float* grad_scale, hipStream_t s) {
  rl_loss_kernel<<<1, 1, 0, s>>>(scal, lm, w, out, grad_scale);
  CAPGEN_HIP(hipGetLastError());
}
void rl_grad(const float* logits, const int32_t* tgt, const int32_t* sample, const float* lse, const float* score,
             const float* count, const float* scal, int B, int L, int V, int pad, float w, void* dl, DType t,
             hipStream_t s) {
  if (t == DType::F32)
    rl_grad_kernel<float><<<B * L, 256, 0, s>>>(logits, tgt, sample, lse, score, count, scal, L, V, pad, w, (float*)dl);
  else
    rl_grad_kernel<bf16><<<B * L, 256, 0, s>>>(logits, tgt, sample, lse, score, count, scal, L, V, pad, w, (bf16*)dl);
  CAPGEN_HIP(hipGetLastError());
}
void rl_export(const int32_t* sample, int n, int64_t* out, hipStream_t s) {
  rl_export_kernel<<<(n + 255) / 256, 256, 0, s>>>(sample, n, out);
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
