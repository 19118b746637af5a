// capgen — row-wise / elementwise / optimizer kernels (launcher interface).
#pragma once
#include "capgen_common.h"
#include "gemm.h"

namespace capgen {

// y = LN(drop(a + a_bias) + res + pe[m % pe_L]) * rowmask          (modules.py:86-90, 114-120)
struct LnFwd {
  int M = 0, d = 0;
  int prio = 0;  // 1: the critical-path kernel raises its waves' issue priority (s_setprio)
  const void* a = nullptr;
  const float* a_bias = nullptr;
  Drop drop{};
  const void* res = nullptr;
  const float* pe = nullptr;
  int pe_L = 1;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  RowMask mask{};
  void* y = nullptr;
  void* v_save = nullptr;  // LN input (post residual add), saved for backward
  float* mean = nullptr;
  float* rstd = nullptr;
  uint64_t* stamp = nullptr;  // diagnostic timestamps (StampScope)
  int wt = -1;                // write-through (sc1) y / v_save stores: 1/0, -1 = wt_default()
};
void layernorm_fwd(const LnFwd& a, DType t, hipStream_t s);

struct LnBwd {
  int M = 0, d = 0;
  int prio = 0;  // as LnFwd::prio
  const void* dy = nullptr;
  const void* v = nullptr;
  const float* mean = nullptr;
  const float* rstd = nullptr;
  const float* gamma = nullptr;
  RowMask mask{};
  Drop drop{};             // the dropout applied to `a` in the forward
  void* d_res = nullptr;   // grad wrt residual input (= grad wrt LN input), or null
  void* d_a = nullptr;     // grad wrt a (dropout mask applied), or null
  float* dgamma = nullptr;  // accumulated
  float* dbeta = nullptr;   // accumulated
  float* dbias = nullptr;   // accumulated column sum of d_a (bias of the producing Linear), or null
  // contention relief: workgroup w accumulates into dgamma/dbeta/dbias + (w % stripes) * stripe_stride
  int stripes = 1;
  int64_t stripe_stride = 0;
  uint64_t* stamp = nullptr;  // diagnostic timestamps (StampScope)
  int wt = -1;                // write-through (sc1) d_res / d_a stores: 1/0, -1 = wt_default()
};
void layernorm_bwd(const LnBwd& a, DType t, hipStream_t s);

// out[m] = [feats[m] | pos[m] | 0] (width Kp), valid[m] = any(pos[m] != 0)  (model.py:202-209)
// img_idx (optional, [M/N]): rows of image img_idx[b] of a resident [n_img, N, F] / [.., P] store
// (indices outside [0, n_img) give all-padding rows)
void pack_encoder_input(const void* feats, DType feats_t, const float* pos, int M, int F, int P, int Kp,
                        void* out, DType out_t, uint8_t* valid, hipStream_t s, const int32_t* img_idx = nullptr,
                        int N = 0, int n_img = 0, uint64_t* seed_bump = nullptr);
// caps [B][T] -> ids_in [B][T-1], tgt [B][T-1]; count = #(tgt != pad) as f32   (model.py:88-89);
// inv_count (optional): 1 / count, the CE mean's gradient scale (model.py:96)
void prepare_captions(const int32_t* caps, int B, int T, int pad, int32_t* ids_in, int32_t* tgt,
                      float* count, hipStream_t s, uint64_t* seed_bump = nullptr, float* inv_count = nullptr);
// out[m] = table[ids[m]] (f32 table -> T)                                      (model.py:432)
// (table_rows: rows of the table, for the hazard checker's byte ranges only)
void embedding_gather(const float* table, const int32_t* ids, int64_t ids_ld, int M, int d, void* out, DType t,
                      hipStream_t s, int64_t table_rows = 0);
// grad[ids[m]] += dE[m] for ids[m] != pad  (nn.Embedding padding_idx)
void embedding_scatter_add(const void* dE, const int32_t* ids, int M, int d, int pad, float* grad, DType t,
                           hipStream_t s, int64_t table_rows = 0);
// db[n] += alpha (* *alpha_ptr) * sum_m X[m][n]
void column_sum(const void* X, int M, int N, int64_t ldx, float alpha, const float* alpha_ptr, float* db,
                DType t, hipStream_t s, int stripes = 1, int64_t stripe_stride = 0);
// dst[i] (+)= sum_s S[s * stride + i], i < n  (folds striped partial sums); clear: the partials
// are zeroed as they are read (the next backward then needs no memset of them)
void stripe_reduce(float* S, int stripes, int64_t stride, int64_t n, float* dst, int accumulate,
                   hipStream_t s, int clear = 0);
// per-row cross entropy: loss_row[m] = lse - logit[tgt], dlogits = softmax - onehot (unscaled, 0 for pad)
void cross_entropy_rows(const float* logits, const int32_t* tgt, int M, int V, int pad, float* loss_row,
                        void* dlogits, DType t, hipStream_t s);
// fused classifier + CE, second half: dl holds exp(v - slab max) from the classifier GEMM's CE
// epilogue (GemmArgs::ce_stats); writes loss_row and rewrites dl as softmax - onehot (0 for pad)
void ce_finish(const float2* stats, int64_t ld, const float* tlogit, const int32_t* tgt, int M, int V, int pad,
               float* loss_row, bf16* dl, hipStream_t s);
// loss = sum(loss_row)/count (or FocalLoss of it); grad_scale = dloss/d(logit sums).
// ce_in: the mean CE is given (all-reduced partials); partial: write sum(loss_row)/count only;
// grad_scale null: the loss only (the scale was written elsewhere, e.g. by prepare_captions).
void loss_finalize(const float* loss_row, int M, const float* count, int focal, float* loss_out,
                   float* grad_scale, hipStream_t s, const float* ce_in = nullptr, int partial = 0);
// Adam (torch.optim.Adam semantics).  step_buf: int64 step counter (incremented here).
void adam_prepare(int64_t* step, float lr, float b1, float b2, float* scal, hipStream_t s);
// Ranges of the shadow (relative to p, element offsets) that adam_update also writes in the fused
// attention fronts' tiled layout (qkv_tile_weights) -- whole 16-row blocks of 512-wide rows
struct AdamTiles {
  static constexpr int kMax = 4;
  int n = 0;
  int64_t off[kMax] = {};
  int64_t len[kMax] = {};
  bf16* dst[kMax] = {};
};
void adam_update(float* p, const float* g, float* m, float* v, size_t n, float b1, float b2, float eps,
                 const float* scal, bf16* shadow, size_t n_shadow, hipStream_t s, int grid_cap = 0,
                 const AdamTiles& tiles = AdamTiles{});
void to_bf16(const float* src, bf16* dst, size_t n, hipStream_t s);
// exact, order-independent checksum of an f32 arena (sum of bit patterns x (2 i + 1) mod 2^64); synchronous
uint64_t arena_checksum(const float* p, size_t n, hipStream_t s);
// greedy: out token = argmax(softmax(logits[b])) (first index on ties)   (model.py:126-128)
void argmax_softmax(const float* logits, int B, int V, int64_t* ids_out, int64_t ids_ld, int col,
                    int32_t* next_ids, int64_t next_ld, hipStream_t s, int logsm = 0);
// one beam-search step (model.py:183-190): rows j*B + i (j < k_in) of logits [k_in*B][V]; the
// k best (prev[j*B+i] + softmax or log-softmax (logsm) of row j*B+i at v) per image i ->
// out_prob/src/tok[sel*B + i]; cand_v/cand_i: k_in*B*k scratch (each row's k finalists)
void beam_step_topk(const float* logits, const float* prev, int k_in, int B, int V, int k, int logsm, float* cand_v,
                    int32_t* cand_i, float* out_prob, int32_t* out_src, int32_t* out_tok, hipStream_t s);
// bf16 decode selection from the classifier epilogue's slab stats (GemmArgs::dec_stats: {max,
// sum exp(v - max)} per row and 16-column slab, stats row stride S = ceil(V / 16)):
// greedy -- argmax of the logits (first index on ties), read from the best slab only;
// beam -- each row's k best scores from its k best slabs (every top-k element lies in the k
// slabs with the largest maxima under (max desc, slab asc)), then the per-image merge.
// V <= 16384 (S <= 1024 slabs, 16 per lane in registers).
bool slab_select_ok(int V);
void slab_argmax(const float* logits, const float2* stats, int B, int V, int64_t* ids_out, int64_t ids_ld, int col,
                 int32_t* next_ids, int64_t next_ld, hipStream_t s);
// the bf16 beam step of every image in one launch (slab selection + merge + the reorder of the sequences,
// ids and K/V row table into the *_dst buffers, chosen token at column t + 1; ops.hip)
void beam_slab_step(const float* logits, const float2* stats, const float* prev, int k_in, int B, int V, int k,
                    int logsm, float* out_prob, int32_t* out_src, int32_t* out_tok, const int64_t* seq_src,
                    int64_t* seq_dst, int Tw, const int32_t* ids_src, int32_t* ids_dst, const int32_t* kv_src,
                    int32_t* kv_dst, int Tc, int t, hipStream_t s);
void beam_step_topk_slab(const float* logits, const float2* stats, const float* prev, int k_in, int B, int V, int k,
                         int logsm, float* cand_v, int32_t* cand_i, float* out_prob, int32_t* out_src,
                         int32_t* out_tok, hipStream_t s);
void bump_seed(uint64_t* seed, hipStream_t s);

}  // namespace capgen
