/* capgen — C ABI of the MI355X-native caption-generator training engine (libcapgen.so).
 *
 * Drop-in boundary.  The reference has no FFI: its boundary is the
 * Python object API of core/models.py (TRANSFORMER, models.py:81-135) over
 * core/TRANSFORMER/model.py (Transformer, model.py:8-209).  Every entry point below
 * replaces one reference call; the Python mirror (image-caption_amd/capgen) binds them
 * with ctypes and keeps the reference method names, arguments and return types.
 *
 * Conventions: all functions return 0 on success, nonzero on failure, with a
 * thread-local message from capgen_last_error().  Device pointers are plain pointers
 * into the current HIP device's memory; `stream` is a hipStream_t passed as void*
 * (NULL = default stream).  Calls on one handle are not thread-safe and are
 * asynchronous on `stream` unless stated otherwise.  The library owns weights, grads,
 * optimizer state and workspaces; the caller owns input/output buffers.
 */
#ifndef CAPGEN_H
#define CAPGEN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CAPGEN_ABI_VERSION 11

typedef struct capgen_engine capgen_t;

enum capgen_dtype { CAPGEN_F32 = 0, CAPGEN_BF16 = 1 };

/* Model/solver shape.  Field meanings follow Transformer.__init__ (model.py:10-36) and
 * core/config.py:5-62; `max_length` is the Transformer's max_length (the decoder
 * positional table has max_length-1 rows, model.py:383-396). */
typedef struct capgen_config {
  int32_t num_vocab, max_length;
  int32_t dim_features, dim_positions;                 /* ENCODE_DIM_FEATURES / _POSITIONS */
  int32_t enc_d, enc_ff, enc_blocks, enc_heads;        /* encode_input_size(=q_k=v), hidden, blocks, heads */
  int32_t dim_word_embedding;
  int32_t dec_d, dec_ff, dec_blocks, dec_heads;
  float dropout;                                       /* DROPOUT (modules.py:64,106) */
  float attention_dropout;                             /* 0.1, hard-coded at modules.py:8 */
  int32_t pad_idx;                                     /* PAD_IDX */
  int32_t encode_mask;                                 /* ENCODE_MASK (model.py:311-328) */
  int32_t focal_loss;                                  /* 'FocalLoss' in OUTPUT_NAME (model.py:73-76) */
  int32_t split_position;                              /* SPLIT_POSITION (model.py:231-233, 297-303): the
                                                          position Linear split into Linear(4, d) over
                                                          the box columns and Linear(P-4, d) over the
                                                          class columns; the same arena columns, two
                                                          table entries (position_ / object_embedding) */
  int32_t split_image_objects;                         /* SPLIT_IMAGE_OBJECTS (model.py:237-244, 258-292): an
                                                          extra EncoderBlock (encoder.image_encoder) over
                                                          every (image row, region) pair, causal + key-pad
                                                          masked; its region token + the position
                                                          embedding feed the shared encoder norm */
  int32_t move_first_image_feature;                    /* MOVE_FIRST_IMAGE_FAETURE (model.py:400-407,
                                                          451-457): after the last decoder block,
                                                          LN(x + drop(FFN(x + enc_out[:, 0]))) */
  int32_t dtype;                                       /* capgen_dtype: compute/storage of activations */
  int32_t max_batch, max_regions;                      /* workspace sizing hints */
  float lr, beta1, beta2, eps;                         /* torch.optim.Adam (models.py:111-113) */
  uint64_t seed;                                       /* dropout RNG seed */
} capgen_config;

/* One reference state_dict tensor mapped into the packed parameter arena:
 * element (r, c) of the reference tensor lives at arena[offset + r*row_stride + c]. */
typedef struct capgen_param_info {
  char name[96];
  int32_t ndim;
  int64_t rows, cols;   /* 1-D tensors: rows = 1 */
  int64_t offset, row_stride;
} capgen_param_info;

const char* capgen_last_error(void);
int capgen_abi_version(void);
/* Run-time switches (csrc/knobs.cpp): name without the CAPGEN_ prefix (e.g. "FUSED_CE").  The
 * CAPGEN_<NAME> environment sets the process default when the library first asks; this call changes
 * it afterwards (engines read theirs when created).  Non-zero status for an unknown name or a
 * debug-build-only switch in the product library.  *old (may be null) receives the previous value.
 * capgen_debug_build: 1 in libcapgen_debug.so (-DCAPGEN_DEBUG), else 0. */
int capgen_set_knob(const char* name, int value, int* old);
int capgen_debug_build(void);

/* Host-only (no device needed): the parameter table for a config.  Writes up to `cap`
 * entries, sets *count to the total; *arena_elems = arena size in f32 elements. */
int capgen_param_table(const capgen_config* cfg, capgen_param_info* out, int cap, int* count,
                       int64_t* arena_elems);

/* Transformer(...).to(DEVICE) + Adam(...)  — models.py:86-113. */
int capgen_create(const capgen_config* cfg, int device, capgen_t** out);
int capgen_destroy(capgen_t* h);

/* state_dict()/load_state_dict() (models.py:62-68) go through these synchronous host
 * copies of the whole f32 arena (layout: capgen_param_table). */
int capgen_get_params(capgen_t* h, float* host_dst, int64_t n);
int capgen_set_params(capgen_t* h, const float* host_src, int64_t n);  /* also resets nothing else */
int capgen_get_grads(capgen_t* h, float* host_dst, int64_t n);
/* Overwrite the gradient arena (e.g. gradients reduced outside the engine), then capgen_adam_step
 * applies them: the host side of a custom data-parallel reduction. */
int capgen_set_grads(capgen_t* h, const float* host_src, int64_t n);
/* Adam state: step count and exp_avg / exp_avg_sq arenas (optional checkpoint interop). */
int capgen_get_adam_state(capgen_t* h, int64_t* step, float* exp_avg, float* exp_avg_sq, int64_t n);
int capgen_set_adam_state(capgen_t* h, int64_t step, const float* exp_avg, const float* exp_avg_sq, int64_t n);
/* Device pointers of the f32 parameter / gradient arenas (for zero-copy views). */
int capgen_arenas(capgen_t* h, float** params, float** grads, int64_t* n);

/* nn.Module.train()/eval(): dropout on/off (modules.py:12,64,106). */
int capgen_set_training(capgen_t* h, int training);

/* Transformer.forward (model.py:79-98) in training state: saves activations for
 * capgen_backward.  feats [B,N,F] (feats_dtype), pos [B,N,P] f32, caps [B,T] int32, all
 * device pointers.  loss_out: device f32 scalar (NULL = internal). */
int capgen_forward(capgen_t* h, const void* feats, int feats_dtype, const float* pos, const int32_t* caps,
                   int B, int N, int T, float* loss_out, void* stream);
/* loss.backward() (models.py:125): fills the gradient arena (overwrites, = zero_grad + backward). */
int capgen_backward(capgen_t* h, void* stream);
/* optimizer.step() (models.py:126). */
int capgen_adam_step(capgen_t* h, void* stream);
/* TRANSFORMER.train_step (models.py:115-126): forward + backward (+ DP gradient
 * all-reduce) + Adam, replayed from a captured hipGraph after the first call with a
 * given (shape, pointers). */
int capgen_train_step(capgen_t* h, const void* feats, int feats_dtype, const float* pos, const int32_t* caps,
                      int B, int N, int T, float* loss_out, void* stream);
int capgen_set_graph(capgen_t* h, int enable);
/* TRANSFORMER.compute_loss (models.py:128-135): forward under no_grad. */
int capgen_compute_loss(capgen_t* h, const void* feats, int feats_dtype, const float* pos, const int32_t* caps,
                        int B, int N, int T, float* loss_out, void* stream);
/* Logits of the last forward/compute_loss, [B*(T-1), V] f32 device copy (test hook). */
int capgen_copy_logits(capgen_t* h, float* dst, int64_t n, void* stream);

/* Transformer.generate_caption_vector (model.py:101-132): greedy decode, bit-identical
 * to the reference's full-prefix recompute but KV-cached.  ids_out: [B, max_length+1]
 * int64 device; attn_out (nullable): [max_length-1, B, N] f32 device (attention_list). */
int capgen_greedy(capgen_t* h, const void* feats, int feats_dtype, const float* pos, int B, int N,
                  int64_t* ids_out, float* attn_out, void* stream);
/* Transformer.beam_search (model.py:135-200): ids_out [B, max_length] int64 device. */
int capgen_beam(capgen_t* h, const void* feats, int feats_dtype, const float* pos, int B, int N, int beam_size,
                int64_t* ids_out, void* stream);

/* Decode scoring of capgen_greedy / capgen_beam: 0 (default) = Transformer (argmax of Softmax,
 * beams accumulate probabilities, model.py:124-128,183); 1 = PolicyNetwork, the SCST model
 * (argmax of LogSoftmax, beams accumulate log-probabilities, model_RL.py:72,126-127,157,182). */
int capgen_set_decode_log_softmax(capgen_t* h, int enable);

/* Reset the device-side dropout RNG state (test hook: replays a dropout mask). */
int capgen_set_rng_seed(capgen_t* h, uint64_t seed);
/* Kernel test hook: C[M,N] = alpha*opA.opB (+bias)(relu) (+C if beta) with the engine's GEMM.
 * ta: A stored [K][M]; tb: B stored [K][N] (else [N][K]).  in/out dtypes: capgen_dtype. */
int capgen_debug_gemm(int M, int N, int K, const void* A, int64_t lda, int ta, const void* B, int64_t ldb, int tb,
                      void* C, int64_t ldc, int in_dtype, int out_dtype, const float* bias, float alpha, int beta,
                      int relu, void* stream);

/* Kernel test hook for the register-B GEMM (gemm_breg.hip, the bf16 decode step's Linears): writes
 * B's MFMA fragment pieces into Bt (N * K bf16; B stored [K][N] if tb else [N][K]), then
 * C[M,N] = A[M,K] . B (+bias)(relu)(zeroed where aux <= 0)(+C if beta) on that kernel; fails if the
 * shape / epilogue is one the kernel does not take (N % 64, K % 256 -- K % 128 at N >= 1536, M >= 1024). */
int capgen_debug_gemm_tiled(int M, int N, int K, const void* A, int64_t lda, const void* B, int64_t ldb, int tb,
                            void* Bt, void* C, int64_t ldc, int out_dtype, const float* bias, int beta, int relu,
                            const void* aux, int64_t ldaux, void* stream);

/* Kernel test hook for the register-B GEMM with the decode step's folded LayerNorm (K = 512): as
 * capgen_debug_gemm_tiled (tb = 0) with LayerNorm inputs v = A (+ ln_res if non-null; both [M][512]
 * bf16); the kernel multiplies y = ((v - mean) * rstd * ln_gamma + ln_beta) * keep (eps 1e-6; keep = 0
 * for rows m with ln_ids[m * ln_ids_ld] == ln_pad when ln_ids is non-null) and also stores y into ln_y
 * ([M][512] bf16). */
int capgen_debug_gemm_tiled_ln(int M, int N, const void* A, const void* ln_res, const void* B, void* Bt, void* C,
                               int out_dtype, const float* bias, int beta, int relu, const float* ln_gamma,
                               const float* ln_beta, void* ln_y, const int32_t* ln_ids, int64_t ln_ids_ld, int ln_pad,
                               void* stream);

/* Experiment hook: force a GEMM tile/wave/pipeline variant (0 = production heuristic). */
int capgen_debug_gemm_variant(int variant);
/* Diagnostic hook: the in-launch split-K combine's hand-off protocol (0 = the production form:
 * sc1 slab stores, agent acquire + plain slab loads in the combining workgroup, tickets re-armed
 * by the last arriver's atomic exchange).  Bits: 1 adds a writer release fence, 2 drops the
 * reader acquire, 4 reads the slabs with sc1 loads, 8 zeroes the tickets with a memset before
 * every launch, 16 re-arms tickets with a relaxed atomic store (round 1 = 2|4|16;
 * tools/splitk_stress.py, tools/step_det_probe.py). */
int capgen_debug_splitk_protocol(int proto);
/* Diagnostic: split-K hand-off counters collected under protocol bit 64 (out4[0] = tickets found
 * out of range at arrival, out4[1] = tiles combined); synchronises the device; reset != 0 zeroes. */
int capgen_debug_splitk_diag(int* out4, int reset);
/* Diagnostic (GEMM ablation build only, protocol bit 4096): device buffer (>= 88 u64) that block 0 of
 * the next GEMM launches fills with per-phase s_memtime / s_memrealtime stamps (gemm_bf16.hip ABL_T). */
int capgen_debug_gemm_timing_buf(void* dev_buf);
/* Diagnostic: synchronous copy of an internal buffer to host: 0 tmp, 1 gOut, 2 gRes, 3 cross-K/V
 * gradient, 4-7 the last encoder block's FFN-hidden / FFN-LN / MHA-LN / QKV gradients; 32 + 8 l + j
 * encoder block l's gAf / gH / gA1 / gATT1 / gQKV; 80 + l the encoder activations X[l]; 128 + 8 l + j
 * encoder block l's saved forward tensors (att, v1, m1, r1, Y, v2, m2, r2); 200 + l / 216 + l the
 * encoder / decoder block l's FFN hidden activations (relu output, the backward's ReLU mask). */
int capgen_debug_copy_buffer(capgen_t* h, int which, void* host_dst, int64_t bytes);

/* Training step over an HBM-resident feature store (replaces TrainDataset.__getitem__ + the
 * DataLoader collate + `.to(DEVICE)`, dataset.py:12-18, main.py:37-43, models.py:120-122):
 * feat_store [n_images, N, F] and pos_store [n_images, N, P] stay on the device (a COCO split in
 * bf16 is ~17 GB); img_idx [B] (device int32) selects each caption's image, gathered inside the
 * encoder-input pack kernel; caps [B, T] device int32.  Otherwise as capgen_train_step. */
int capgen_train_step_indexed(capgen_t* h, const void* feat_store, int feats_dtype, const float* pos_store,
                              int n_images, const int32_t* img_idx, const int32_t* caps, int B, int N, int T,
                              float* loss_out, void* stream);

/* Self-critical sequence training (SelfCriticNetwork, models.py:137-211), in two calls with the
 * host scoring the samples in between (CIDEr-D / BLEU, capgen/scst.py):
 *  capgen_rl_sample  replaces PolicyNetwork.forward + .sample (model_RL.py:75-97) and the entropy
 *                    of StructureCriterion (loss.py:123-127): teacher-forced forward (dropout as
 *                    set by capgen_set_training), sample = argmax log_softmax [B, T-1] (int64),
 *                    per-image masked mean entropy [B] and the CrossEntropy LM loss [1];
 *  capgen_rl_finish  replaces ReinforcementLearningLoss.forward (loss.py:53-76, 131-152) and, when
 *                    train != 0, loss.backward() + Adam.step() (models.py:191-195).  scores [B]
 *                    (device) = per-image total score (cider_w*CIDEr-D + bleu_w*BLEU-4 +
 *                    entropy_w*entropy + self_cider_w*self-CIDEr); loss_out [3] (device) =
 *                    {loss, language_model_loss, structure_loss}.  Under DP, sum(mask) and the
 *                    structure numerator are all-reduced (global mean as in one process). */
int capgen_rl_sample(capgen_t* h, const void* feats, int feats_dtype, const float* pos, const int32_t* caps, int B,
                     int N, int T, int64_t* sample_out, float* entropy_out, float* lm_loss_out, void* stream);
int capgen_rl_finish(capgen_t* h, const float* scores, float structure_loss_weight, float* loss_out, int train,
                     void* stream);

/* Host rewards for self-critical training, natively (StructureCriterion.get_scores,
 * loss.py:154-181, as restated by capgen/scst.py): out[b] = cider_w * CIDEr-D(sample_b | target_b)
 * + bleu_w * BLEU-4(sample_b | target_b), CIDEr-D with document frequencies from the B targets
 * (coco-caption 'corpus' mode, sigma 6, x10), per-sentence BLEU-4 with coco-caption smoothing.
 * target / sample: host int64 [B][L] token ids (row strides target_ld / sample_ld), read as
 * decode_captions does (core/utils.py:67-103): <START> at t = 0 skipped, <END> ends the sentence
 * as the token dot_id ("."; pass -1 when the vocabulary has no "." word), <NULL> dropped.
 * Pure host code: no device, no handle. */
int capgen_scst_rewards(const int64_t* target, int64_t target_ld, const int64_t* sample, int64_t sample_ld, int B,
                        int L, int start_id, int end_id, int null_id, int64_t dot_id, double cider_w, double bleu_w,
                        double* out);

/* Test hook: one masked multi-head attention forward (+ backward when dout != NULL) on packed
 * [B, L, H*dk] tensors (row stride H*dk), dtype 0 = f32, 1 = bf16 (the kernels the engine uses
 * for modules.py:16-27 ScaledDotProductAttention).  key_valid: optional [B][Lk] bytes (0 =
 * masked key); causal masks keys j > i.  probs: optional [B,H,Lq,Lk] f32 output. */
int capgen_debug_attention(int dtype, int B, int H, int Lq, int Lk, int dk, const void* q, const void* k,
                           const void* v, const unsigned char* key_valid, int causal, float temperature, void* o,
                           float* probs, const void* dout, void* dq, void* dk_, void* dv, void* stream);

/* Test hook: the fused self-attention front (qkv_attn.hip; modules.py:67-76 then 16-27), bf16:
 * qkv [B*L, 3*H*64] = X [B*L, H*64] . W^T (W = [q; k; v] weights [3*H*64, H*64]), then the masked
 * attention of every (image, head) into o [B*L, H*64].  key_valid [B][L] bytes / key_ids [B][L]
 * int32 (== pad_idx: masked) optional; causal masks keys j > i.  Head size 64, H*64 = 512 only. */
int capgen_debug_qkv_attention(int B, int L, int H, const void* X, const void* W, void* qkv, void* o,
                               const unsigned char* key_valid, const int32_t* key_ids, int pad_idx, int causal,
                               void* stream);

/* Test hook: the fused cross-attention front (qkv_attn.hip cross mode; modules.py:195-197), bf16:
 * q [B*Lq, H*64] = X . Wq^T, then attention over K / V = KV [B*Lk, 2*H*64] (k | v per row) with the
 * key mask key_valid [B][Lk] (optional) into o [B*Lq, H*64].  Head size 64, H*64 = 512 only. */
int capgen_debug_cross_attention(int B, int Lq, int Lk, int H, const void* X, const void* Wq, const void* KV, void* q,
                                 void* o, const unsigned char* key_valid, void* stream);

/* Test hook: the fused output side of an attention block's backward (qkv_attn.hip qkv_attn_bwd;
 * modules.py:77 o_linear + 16-27), bf16: dO = dA . Wo (dA [B*Lq, 512], Wo [512, 512] nn.Linear), then
 * the masked attention backward over packed q [B*Lq, 512], k / v [B*Lk, 512] (key_valid [B][Lk]
 * optional, causal) into dq / dk / dv.  Head size 64, H * 64 = 512. */
int capgen_debug_attention_bwd_wo(int B, int Lq, int Lk, int H, const void* q, const void* k, const void* v,
                                  const unsigned char* key_valid, int causal, const void* dA, const void* Wo, void* dq,
                                  void* dk, void* dv, void* stream);

/* Persisted GEMM autotune table (no reference counterpart: the reference's GEMMs are cuBLAS calls
 * of torch eager, models.py:120-126).  The bf16 GEMM picks a tile / wave / pipeline / split-K
 * variant per shape by timing; a table file fixes those choices so that every process (bench,
 * tests, profiles) runs the same kernels.  load merges a file (returns the entries read, or -1:
 * no file); save writes every choice known to this process; tune_live_count = shapes this
 * process had to tune itself (a complete table keeps it 0).  libcapgen loads
 * $CAPGEN_TUNE_TABLE (default: tune_gfx950.txt next to the library) at first use. */
int capgen_tune_load(const char* path);
int capgen_tune_save(const char* path);
int capgen_tune_live_count(void);

/* Diagnostics of the multi-stream step (hazard.h): op 1 = start logging every launch's stream and
 * device byte ranges and every event / host-sync edge (clears the log), 0 = stop, 2 = check the log:
 * *n_conflicts = unordered pairs of launches on different streams touching overlapping bytes (at
 * least one writing), report (cap bytes, NUL-terminated) = the first of them.  side_delay: a spin
 * kernel of `us` microseconds in front of every launch off the critical stream (0 = off). */
int capgen_debug_hazard(int op, char* report, int cap, int* n_conflicts);
int capgen_debug_side_delay(double us);
/* The engine's RCCL call sequence (op 1 = start recording + clear, 0 = stop, 2 = dump one line per
 * collective: name, bytes, stream role).  Every rank must issue the identical sequence whatever its
 * batch, or the ranks deadlock (test hook for the data-parallel step). */
int capgen_debug_collectives(capgen_t* h, int op, char* out, int cap);
/* Un-profiled per-kernel timeline: op 1 = give every GEMM / LayerNorm / attention launch of the
 * following steps a timestamp slot (drops the captured forward so it re-captures with them), 3 = arm
 * (zero the slots; device synchronised), 2 = read: out[2i], out[2i+1] = start / end (us, 100 MHz
 * real-time counter) of slot i of the last step, names = one line per slot ("crit|side|bucket
 * kernel shape"); returns the slot count (-1: error), 0 = off. */
int capgen_debug_stamps(capgen_t* h, int op, double* out, int cap, char* names, int names_cap);

/* Data parallel (one process per GPU, RCCL over xGMI).  Rank 0 creates the 128-byte
 * unique id; the host broadcasts it (torch.distributed store) and every rank calls
 * capgen_dp_init, which also broadcasts rank 0's parameters. */
int capgen_dp_unique_id(char out[128]);
int capgen_dp_init(capgen_t* h, const char id[128], int rank, int world);
/* Override the global non-pad target count used by the CE mean (<= 0: all-reduce it).  Waits for
 * the previous step's copy of the override (no race with an in-flight step).  Under DP every rank's
 * loss output is the GLOBAL mean (Focal) loss: the per-rank partial CE sums are all-reduced before
 * the FocalLoss transform and the gradient scale (model.py:73-76, loss.py:20-28). */
int capgen_dp_set_global_count(capgen_t* h, float count);

/* Sharded parameter update (ZeRO-1; replaces the per-bucket all-reduce + full Adam that
 * torch.optim.Adam.step over DDP-averaged gradients would be, core/models.py:111-113,124-125).
 * With world > 1 (default; CAPGEN_ZERO=0 disables) every gradient bucket is reduce-scattered,
 * each rank runs Adam on its 1/world chunk, and the updated f32 chunk is all-gathered in place.
 * Parameters stay replicated on every rank after each step; the Adam moments are current only
 * in this rank's chunks -- capgen_dp_sync_adam_state (collective, every rank) all-gathers them
 * before capgen_get_adam_state is used for a checkpoint.
 * capgen_dp_buckets: the last train step's bucket ranges [off, off + count) over the parameter
 * arena, in issue order (rank r owns [off + r*count/world, off + (r+1)*count/world) of each).
 * capgen_dp_debug_shard (test hook): without any collective, update as rank `rank` of `world`
 * would (Adam on this rank's chunks only); world <= 1 turns it off. */
int capgen_dp_sync_adam_state(capgen_t* h);
/* The engine communicator's size and this rank (ncclCommCount / ncclCommUserRank; 0 / 0 before
 * capgen_dp_init).  At world > 1 the FIRST capgen_train_step / capgen_train_step_indexed also checks,
 * once, that every rank holds the same global non-pad count and loss (max == min over the ranks; the
 * loss the step wrote to loss_out, or its internal loss when loss_out was null) and fails the step
 * otherwise.  capgen_dp_check runs that same exchange now, at any world size (collective: every rank
 * calls it; needs capgen_dp_init and a train step before it; loss null = the buffer the last forward
 * wrote its loss to) -- the world-1 rehearsal of the check. */
int capgen_dp_comm_info(capgen_t* h, int* nranks, int* rank);
int capgen_dp_check(capgen_t* h, const float* loss, void* stream);
/* Exact, order-independent checksum of the f32 parameter arena (sum of the bit patterns times
 * (2 i + 1), mod 2^64; synchronous): equal parameters give equal values on every rank. */
int capgen_params_checksum(capgen_t* h, uint64_t* out);
int capgen_dp_buckets(capgen_t* h, int64_t* offs, int64_t* counts, int cap, int* n);
int capgen_dp_debug_shard(capgen_t* h, int rank, int world);

#ifdef __cplusplus
}
#endif
#endif /* CAPGEN_H */
