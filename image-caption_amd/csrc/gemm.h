// capgen — GEMM launcher interface (see gemm.hip for the kernel).
#pragma once
#include <type_traits>

#include "capgen_common.h"

namespace capgen {

enum class DType : int { F32 = 0, BF16 = 1 };

inline size_t dsize(DType t) { return t == DType::F32 ? 4 : 2; }

// (explicit pad_ fields: no implicit padding, so a GemmArgs / GemmGroup is fully described by its
// bytes -- the grouped launch's device-resident argument table keys on them)
struct GemmArgs {
  int M = 0, N = 0, K = 0, pad0_ = 0;
  const void* A = nullptr;
  int64_t lda = 0;
  const void* B = nullptr;
  int64_t ldb = 0;
  void* C = nullptr;
  int64_t ldc = 0;
  const float* bias = nullptr;      // [N] f32, added before relu
  const void* aux = nullptr;        // same dtype as A/B: zero the output where aux[m][n] <= 0
  int64_t ldaux = 0;
  float alpha = 1.f;
  int pad1_ = 0;
  const float* alpha_ptr = nullptr;  // device scalar multiplied into alpha (e.g. 1/count)
  int beta = 0;                      // 1: accumulate into C
  int prio = 0;                      // 1: critical-path launch, waves raise their issue priority
  const void* bt = nullptr;          // bf16: B's MFMA fragment pieces (gemm_tile_b) -> the register-B
  int64_t bt_pad_ = 0;               //   path (gemm_breg.hip) where it takes the shape; null: the LDS ring
  void* C2 = nullptr;                // bf16 path: columns n >= nsplit go to C2[m][n - nsplit] (row
  int64_t ldc2 = 0;                  //   stride ldc2), e.g. Q to one buffer and K/V to a cache
  int nsplit = 0;                    //   (nsplit % 4 == 0)
  int relu = 0;
  float* colsum = nullptr;           // += column sums of the (post-epilogue, beta=0) output, f32 [N]
  int colsum_stripes = 1;            // workgroup w adds into colsum + (w % stripes) * colsum_stride
  int pad2_ = 0;
  int64_t colsum_stride = 0;
  // fused cross-entropy epilogue (bf16 NT path only; classifier + CE, model.py:93-96): per row m
  // and 16-column slab c, v = alpha * acc + bias, mx = max(v), C[m][n] = exp(v - mx) (bf16) and
  // ce_stats[m * ce_ld + c] = {mx, sum exp(v - mx)}; ce_tlogit[m] = v[ce_tgt[m]] (f32).  The
  // logits themselves are never written; ce_finish() turns C into softmax - onehot in place.
  float2* ce_stats = nullptr;
  int64_t ce_ld = 0;
  const int32_t* ce_tgt = nullptr;
  float* ce_tlogit = nullptr;
  // decode classifier epilogue (bf16 operands, f32 out): C[m][n] = v = alpha * acc + bias as usual,
  // plus dec_stats[m * dec_ld + c] = {max, sum exp(v - max)} of each 16-column slab c -- the
  // beam / greedy selection then reads 1/8 of the row (ops.hip slab_topk / slab_argmax)
  float2* dec_stats = nullptr;
  int64_t dec_ld = 0;
  uint64_t* stamp = nullptr;  // diagnostic timestamps (capgen_common.h StampScope); grouped: p[0]'s
  int wt = -1;                // write-through (sc1) C stores (bf16 path): 1/0, -1 = wt_default()
  int pad3_ = 0;
  // LayerNorm folded into the consumer (register-B path, K = 512; the decode step): the LayerNorm
  // input is v = A (+ ln_res, bf16 [M][K]), the kernel multiplies
  // y = ((v - mean) * rstd * ln_gamma + ln_beta) * keep (keep = 0 for rows m with
  // ln_ids[m * ln_ids_ld] == ln_pad when ln_ids is set; modules.py:86-90, 114-120), and the workgroups
  // of column tile 0 also store y into ln_y ([M][K] bf16; neither A nor ln_res)
  const float* ln_gamma = nullptr;
  const float* ln_beta = nullptr;
  void* ln_y = nullptr;
  const int32_t* ln_ids = nullptr;
  int64_t ln_ids_ld = 0;
  int ln_pad = 0;
  int a_table_rows = 0;  // a_ids: rows of the table A (the kernel clamps ids into it; hazard checker)
  const void* ln_res = nullptr;
  // register-B path: A rows gathered by index -- row m of the product is A[a_ids[m * a_ids_ld]] (the
  // decode step's word-embedding projection reads the bf16 embedding table directly)
  const int32_t* a_ids = nullptr;
  int64_t a_ids_ld = 0;
};
// 4 ints + 37 eight-byte fields (pointers, int64s, int/float pairs): the size leaves no room for padding
static_assert(sizeof(GemmArgs) == 16 + 37 * 8, "GemmArgs must have no padding");

// Independent GEMMs of one layout launched as ONE grid (tiles problem after problem).
constexpr int kMaxGroup = 8;
struct GemmGroup {
  int n = 0;
  int start[kMaxGroup + 1] = {};  // first tile of problem i
  int tiles_n[kMaxGroup] = {};    // column tiles of problem i
  GemmArgs p[kMaxGroup];
};
static_assert(sizeof(GemmGroup) == 4 * (1 + 2 * kMaxGroup + 1) + kMaxGroup * sizeof(GemmArgs), "GemmGroup must have no padding");

// ta: A stored [K][M] (else [M][K]); tb: B stored [K][N] (else [N][K]).
void gemm(const GemmArgs& g, DType in, DType out, bool ta, bool tb, hipStream_t s);
// gemm_breg.hip: the bf16 GEMM reading B from its fragment pieces g.bt (A stored [M][K]).
// gemm_tile_b writes the pieces of B (stored [N][K] for tb = 0, [K][N] for tb = 1; N % 16 == 0,
// K % 32 == 0) into Bt (N * K bf16): piece (j, ks) = 512 bf16, lane l holding B[32 ks + 8 (l >> 4) + e]
// [16 j + (l & 15)] for e = 0..7.
bool gemm_breg_ok(const GemmArgs& g);
void gemm_breg(const GemmArgs& g, DType out, hipStream_t s);
void gemm_tile_b(const bf16* B, int64_t ldb, int tb, int N, int K, bf16* Bt, hipStream_t s);
// allocate the per-device zero page used for out-of-range tiles (call before any bf16 gemm,
// outside graph capture)
void gemm_init();
// experiment hook: force a bf16 GEMM tile/wave/stage variant (0 = heuristic)
void gemm_set_variant(int v);
// diagnostic: split-K hand-off protocol bits (0 = the full recipe; gemm_bf16.hip g_splitk_proto)
void gemm_set_splitk_protocol(int p);
// diagnostic (ablation build, protocol bit 4096): device buffer of >= 88 u64 for the phase timestamps
void gemm_set_timing_buf(uint64_t* p);
// diagnostic: read (and optionally zero) the split-K hand-off counters (protocol bit 64)
void gemm_splitk_diag(int* out4, bool reset);
// n <= kMaxGroup independent bf16-operand GEMMs of one layout / output type in one launch
// (tile variant autotuned per group signature); no beta/colsum/alpha_ptr-free restrictions
void gemm_grouped(const GemmArgs* probs, int n, DType out, bool ta, bool tb, hipStream_t s);
// bf16-operand path (gemm_bf16.hip); called by gemm() after argument checks
void gemm_bf16(const GemmArgs& g, DType out, bool ta, bool tb, hipStream_t s);

// Persisted autotune table (gemm_bf16.hip): one line per tuned shape / grouped signature.
// load: merges the file's choices (entries already tuned in this process win); returns the
// number of entries read (-1: no such file).  save: writes every choice made or loaded so far.
int gemm_tune_load(const char* path);
int gemm_tune_save(const char* path);
// number of GEMM shapes autotuned live in this process (a complete table keeps it at 0)
int gemm_tune_live_count();

}  // namespace capgen
