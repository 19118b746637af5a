// capgen — the training/decoding engine behind the C ABI (include/capgen.h).
//
// One engine = one (process, device).  It owns the packed f32 parameter arena (+ bf16
// shadow for the MFMA path), the gradient arena, Adam moments and every activation
// buffer, and sequences the hot path as explicit forward/backward kernel launches on
// its own HIP stream — no autograd, no tracing compiler.  A train step is captured once
// per (shape, input pointers) into a hipGraph and replayed.
//
// Reference call stack restated: models.py:115-126 train_step ->
// model.py:79-98 forward -> Encoder (model.py:294-332) -> EncoderBlock (modules.py:146-157)
// -> Decoder (model.py:419-459) -> DecoderBlock (modules.py:185-206) -> classifier + CE
// (model.py:93-96) -> autograd backward -> Adam.step.
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <vector>

#include "../../include/capgen.h"
#include "attention.h"
#include "gemm.h"
#include "hazard.h"
#include "layout.h"
#include "ops.h"
#include "qkv_attn.h"
#include "variants.h"
#include "rl.h"

using namespace capgen;

namespace {

thread_local std::string g_last_error;

#define NCCL_CHECK(expr)                                                                             \
  do {                                                                                               \
    ncclResult_t _r = (expr);                                                                        \
    if (_r != ncclSuccess) throw Error(std::string(#expr) + ": " + ncclGetErrorString(_r));          \
  } while (0)

// bump allocator: a dry run (base == nullptr) sizes the block, the second run assigns pointers
struct Planner {
  char* base = nullptr;
  size_t used = 0;
  void* raw(size_t bytes) {
    size_t off = (used + 255) & ~size_t(255);
    used = off + bytes;
    return base ? base + off : nullptr;
  }
  template <class P>
  void take(P*& p, size_t count) {
    p = (P*)raw(count * sizeof(P));
  }
};

struct EncAct {
  void *qkv, *att, *v1, *Y, *H, *v2;
  float *P, *m1, *r1, *m2, *r2;
};
struct DecAct {
  void *qkv, *atts, *vs, *D1, *qc, *attc, *vc, *D2, *H, *vf;
  float *Ps, *ms, *rs, *Pc, *mc, *rc, *mf, *rf;
};


struct Acts {
  int B = 0, N = 0, T = 0;  // capacity
  // encoder
  void* Aenc;
  uint8_t* valid;
  void* ev0;
  float *em0, *er0;
  std::vector<void*> X;
  std::vector<EncAct> enc;
  void* KV;
  // decoder
  int32_t *ids, *tgt;
  float* count;
  void* E;
  void* dv0;
  float *dm0, *dr0;
  std::vector<void*> D;
  std::vector<DecAct> dec;
  float* logits;
  void* dlogits;
  float2* ce_stats;  // fused classifier + CE (bf16): {max, sum exp} per row and 16-column slab
  float* ce_tl;      // its target logits
  float *loss_row, *grad_scale, *loss, *loss_ce;
  void* gEnc;     // encoder-chain residual gradient while decoder block 0 finishes on es2 (overlap_dec0)
  // SCST (rl.hip): per-row sample / lse / logp[sample] / entropy, per-image entropy, scalars
  int32_t* rl_sample;
  float *rl_lse, *rl_logp, *rl_ent, *rl_ent_img, *rl_score, *rl_scal;
  // scratch / backward.  gOut/gRes carry the residual-stream gradient (critical path);
  // every other gradient buffer is per block, so the weight-gradient GEMMs that read them can
  // run later on the side stream without a write-after-read hazard.
  void *tmp, *gOut, *gRes, *gKV, *gE, *gAe, *gAd;
  void* tmpf;  // the decoder front's GEMM -> LayerNorm scratch (runs on es2 beside the encoder)
  struct GradBufs {
    void *gAf, *gH, *gA1, *gATT1, *gQKV, *gA2, *gATT2, *gQc;
  };
  std::vector<GradBufs> genc, gdec;
  // split_image_objects (model.py:258-292): the image block runs over 2*B*N pair rows
  void *siY, *siEp, *siX2, *siZ, *siV, *siG0, *siG1, *siGY, *siGEp;
  uint8_t* siValid;
  float *siM, *siR;
  EncAct si;
  GradBufs gsi;
  // move_first_image_feature (model.py:451-457): U = D + enc[:, 0], H, LN output
  void *mfU, *mfH, *mfV, *mfOut, *mfGA, *mfGH, *mfGU;
  float *mfM, *mfR;
};

struct GenWS {
  int R = 0, N = 0;  // capacity (rows, regions)
  void *x, *x1, *x2, *q, *att, *tmp, *h, *E;
  float *mean, *rstd, *Pc, *logits;
  float2* dstats;         // bf16 decode: classifier slab stats [R][ceil(V/16)] (GemmArgs::dec_stats)
  float* cand_v;          // beam: each row's k finalists (beam_step_topk)
  int32_t* cand_i;
  void* cache;            // [Ld][R][Tcap][2d]: row r's K/V of position t at [l][r][t]
  int32_t *ids, *ids2;    // [R][Tcap]
  int32_t *kvrow, *kvrow2;  // beam: [R][Tcap] row holding the K/V of (beam row, position)
  int64_t *seq, *seq2;   // beam [R][Tw]
  float *bprob, *bprob2;
  int32_t *bsrc, *btok;
  int64_t* out_ids;  // staged outputs of a graph-replayed decode: ids [R][maxlen + 1]
  float* out_attn;   // greedy attention_list [maxlen - 1][R][N]
};

__global__ void init_gen_ids_kernel(int64_t* out, int rows, int width, int32_t* ids, int tcap) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < rows * width) out[c] = (c % width) == 0 ? 1 : 0;
  if (c < rows * tcap) ids[c] = (c % tcap) == 0 ? 1 : 0;
}

// dst row r = (j, i) <- src row (src[j][i], i); then optionally set column `col` to tok
template <typename E>
__global__ void beam_gather_kernel(const E* __restrict__ src, E* __restrict__ dst, int64_t row_elems,
                                   int64_t copy_elems, const int32_t* __restrict__ bsrc, int B, int R,
                                   const int32_t* __restrict__ tok, int col) {
  const int r = blockIdx.y;
  const int srow = bsrc[r] * B + (r % B);
  const E* s = src + (int64_t)srow * row_elems;
  E* d = dst + (int64_t)r * row_elems;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < copy_elems; c += (int64_t)gridDim.x * blockDim.x)
    d[c] = (tok && c == col) ? (E)tok[r] : s[c];
}

// beam reorder of the K/V row table (attention kv_row): row r's positions 0..t come from its
// source beam's row, position t + 1 (written by row r's own next decoder step) is row r
__global__ void beam_kvrow_kernel(const int32_t* __restrict__ src, int32_t* __restrict__ dst, int Tc, int t,
                                  const int32_t* __restrict__ bsrc, int B, int R) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= R * Tc) return;
  const int r = e / Tc, c = e % Tc;
  const int srow = bsrc[r] * B + (r % B);
  dst[e] = c <= t ? src[(int64_t)srow * Tc + c] : (c == t + 1 ? r : 0);
}

}  // namespace

struct capgen_engine {
  capgen_config cfg;
  Layout L;
  int device = 0;
  DType act = DType::BF16;
  hipStream_t es = nullptr;   // engine stream (critical path)
  hipStream_t es2 = nullptr;  // side stream: weight-gradient GEMMs
  hipStream_t ec = nullptr;   // bucket stream: per-bucket gradient all-reduce (RCCL) + Adam
  hipEvent_t ev_in = nullptr, ev_out = nullptr, ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_b1 = nullptr, ev_b2 = nullptr, ev_cj = nullptr;
  hipEvent_t ev_ff = nullptr, ev_fj = nullptr;  // forward: decoder front forked to / joined from es2
  float *params = nullptr, *grads = nullptr, *am = nullptr, *av = nullptr;
  bf16* shadow = nullptr;
  // the fused attention fronts' weights (every self-attention Wqkv, every cross Wq) in the tiled
  // layout of qkv_tile_weights, re-tiled from the shadow wherever the shadow is written
  bf16* wtile = nullptr;
  // arena offset -> (element offset in wtile, rows); rows < 0: an output projection Wo [512][512]
  // kept as the tiled Wo^T (the fused attention backward's dO = dA . Wo[:, head], qkv_attn_bwd)
  std::map<int64_t, std::pair<int64_t, int>> tiled;
  const bf16* WT(int64_t woff) const {
    auto it = tiled.find(woff);
    return it == tiled.end() || it->second.second < 0 ? nullptr : wtile + it->second.first;
  }
  const bf16* WTo(int64_t woff) const {
    auto it = tiled.find(woff);
    return it == tiled.end() || it->second.second > 0 ? nullptr : wtile + it->second.first;
  }
  void build_tiles() {  // (bf16 engines, at creation: model widths of 512 only)
    std::vector<std::pair<int64_t, int>> ws;
    if (L.d == 512) {
      for (const auto& e : L.enc) ws.push_back({e.Wqkv, 3 * L.d}), ws.push_back({e.Wo, -512});
      if (L.has_img) ws.push_back({L.img.Wqkv, 3 * L.d}), ws.push_back({L.img.Wo, -512});
    }
    if (L.dd == 512)
      for (const auto& e : L.dec)
        ws.push_back({e.Wqkv, 3 * L.dd}), ws.push_back({e.Wq_c, L.dd}), ws.push_back({e.Wo_s, -512}),
            ws.push_back({e.Wo_c, -512});
    int64_t n = 0;
    for (auto& w : ws) tiled[w.first] = {n, w.second}, n += (int64_t)std::abs(w.second) * 512;
    if (n) CAPGEN_HIP(hipMalloc(&wtile, (size_t)n * 2));
  }
  // re-tile the fronts' weights that overlap the arena range [off, off + n) from the shadow (a matrix
  // cut by a range boundary is re-tiled by both ranges' calls; the later one, on the same stream, sees
  // the whole matrix updated)
  // the weight version: bumped at every enqueued change of the bf16 shadow (each one is followed by
  // retile), so the decode tiles are rebuilt only when the weights moved
  uint64_t wver = 1, dtiles_ver = 0;
  void retile(int64_t off, int64_t n, hipStream_t s, bool trans_only = false) {
    ++wver;
    for (auto& kv : tiled)
      if (kv.first < off + n && kv.first + (int64_t)std::abs(kv.second.second) * 512 > off) {
        if (kv.second.second < 0) qkv_tile_weights_t(shadow + kv.first, 512, wtile + kv.second.first, s);
        else if (!trans_only) qkv_tile_weights(shadow + kv.first, kv.second.second, 512, wtile + kv.second.first, s);
      }
  }
  // bf16 decode: the decoder Linears as MFMA fragment pieces for the register-B GEMM (gemm_breg.hip,
  // CAPGEN_BREG_DECODE, default on).  Wqkv / Wq_c are the fronts' tiles (the same layout at K = 512);
  // the others (Wo_s, Wo_c, W1, W2, the word-embedding projection) are rebuilt from the bf16 shadow at
  // the start of every greedy / beam call -- ~30 MB at C4, the weights may have moved since the last one
  bool breg_decode_on = knob(Knob::BregDecode) != 0;
  bf16* dtiles = nullptr;
  std::map<int64_t, int64_t> dtile;  // arena offset -> element offset in dtiles
  std::vector<std::array<int64_t, 3>> dtile_list() const {  // {arena offset, rows N, columns K}
    std::vector<std::array<int64_t, 3>> v;
    v.push_back({L.Wel, L.dd, L.dwe});
    for (const auto& e : L.dec)
      v.push_back({e.Wo_s, L.dd, L.dd}), v.push_back({e.Wo_c, L.dd, L.dd}), v.push_back({e.W1, L.fd, L.dd}),
          v.push_back({e.W2, L.dd, L.fd});
    return v;
  }
  bool breg_decode() const { return breg_decode_on && act == DType::BF16; }
  const void* DT(int64_t off) const {
    if (!breg_decode()) return nullptr;
    if (const bf16* t = WT(off)) return t;
    auto it = dtile.find(off);
    return it == dtile.end() || !dtiles ? nullptr : dtiles + it->second;
  }
  bf16* emb_bf = nullptr;  // bf16 decode: the word-embedding table, read by the Wel GEMM through the ids
  bool dtiles_init = false;  // set once: a model whose Linears fit no tile shape allocates nothing, once
  void ensure_dtiles() {  // (outside any capture)
    if (dtiles_init || !breg_decode()) return;
    dtiles_init = true;
    int64_t tot = 0;
    for (const auto& t : dtile_list())
      if (t[1] % 16 == 0 && t[2] % 32 == 0) dtile[t[0]] = tot, tot += t[1] * t[2];
    if (tot) CAPGEN_HIP(hipMalloc(&dtiles, (size_t)tot * 2));
#ifndef CAPGEN_NO_GATHER_FOLD
    // only the tiled word-embedding projection reads the bf16 table
    if (L.dwe % 8 == 0 && dtile.count(L.Wel)) CAPGEN_HIP(hipMalloc(&emb_bf, (size_t)L.V * L.dwe * 2));
#endif
  }
  void build_dtiles(hipStream_t s) {
    if (!dtiles) return;
    // skipped while the tiles match the weights (~0.12 ms per greedy / beam call); a build captured
    // into a graph runs at every replay
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    CAPGEN_HIP(hipStreamIsCapturing(s, &cs));
    const bool capturing = cs != hipStreamCaptureStatusNone;
    if (!capturing && dtiles_ver == wver) return;
    if (!capturing) dtiles_ver = wver;
    if (emb_bf) to_bf16(P(L.emb), emb_bf, (size_t)L.V * L.dwe, s);
    for (const auto& t : dtile_list()) {
      auto it = dtile.find(t[0]);
      if (it != dtile.end()) gemm_tile_b(shadow + t[0], t[2], 0, (int)t[1], (int)t[2], dtiles + it->second, s);
    }
  }
  float* pe = nullptr;  // [max_length-1, dd] f32 sinusoid table
  int64_t* step = nullptr;
  float* adam_scal = nullptr;
  uint64_t* seed = nullptr;
  float* scalars = nullptr;  // internal loss
  // striped partial sums for the small accumulated gradients (LayerNorm gamma/beta, biases):
  // [NSTRIPE][total - enc_lng]; folded into the gradient arena by stripe_reduce
  static constexpr int NSTRIPE = 16;
  float* gstripe = nullptr;
  bool stripes_dirty = true;  // gstripe may hold partials (the next backward zeroes it first)
  bool stripe_clear = knob(Knob::StripeClear) != 0;  // the folds zero the partials they read (0: memset per step)
  int64_t n_small = 0;
  bool training = true;
  bool fwd_drop = true;  // dropout state of the last forward (backward must match)
  int fB = 0, fN = 0, fT = 0;  // shape of the last forward
  Acts a;
  void* ws = nullptr;
  GenWS g;
  void* gws = nullptr;
  // graph: off by default.  Measured on MI355X / ROCm 7 (tools/launch_probe.py): a replay of
  // the three-stream step graph costs ~3 ms of host time and runs ~0.7 ms SLOWER on the GPU
  // than the same kernels issued eagerly on three streams (4.3 vs 5.0 ms at C2); a
  // single-stream graph launches in 0.1 ms but loses the stream overlap (5.5 ms).
  bool graph_on = false;
  hipGraphExec_t gexec = nullptr;
  // eager step mode: the forward alone as a linear graph (CAPGEN_FWD_GRAPH=0 disables)
  // (1: at world size 1 -- its RCCL count / CE all-reduces, if any, capture into the graph; at world > 1
  // the forward is issued eagerly, the collectives as plain stream calls: the multi-rank path keeps
  // RCCL's standard usage, and eager vs graph measured level on the GPU; 2: the graph at any world size)
  int fwd_graph_mode = knob(Knob::FwdGraph);
  bool fwd_graph_on = fwd_graph_mode != 0;
  hipGraphExec_t fexec = nullptr;
  // split forward graphs (CAPGEN_FWD_SPLIT=1, with the decoder front on es2): the front and the
  // critical chain as separate LINEAR graphs on their own streams.  Under rocprofv3 the one
  // multi-stream graph ran its front branch before the encoder (no overlap) and the split graphs
  // overlapped, but without the profiler the single graph measured faster (4-round A/B: 3.032 vs
  // 3.048 ms/step; front off: 3.072).  The multi-branch graph costs the host more to launch
  // (enqueue per step 2.52 vs 2.27 ms; linear graphs ~0.1 us per node), which matters once the
  // step also issues the per-bucket collectives.  The single graph is the default at every world
  // size (faster on the GPU; the count / partial-CE all-reduces capture into it as well);
  // CAPGEN_FWD_SPLIT=1 selects the split graphs
  int fwd_split_env = knob(Knob::FwdSplit);
  bool fwd_split() const { return fwd_split_env == 1; }
  bool cap_split = false;  // forward() is being captured in split mode: it ends/begins captures
  hipGraph_t fg[4] = {};   // pre, front, encoder, decoder
  hipGraphExec_t fx[4] = {};
  void cap_cut(hipStream_t from, int idx, hipStream_t next) {  // end capture on `from` into fg[idx]
    CAPGEN_HIP(hipStreamEndCapture(from, &fg[idx]));
    if (next) CAPGEN_HIP(hipStreamBeginCapture(next, hipStreamCaptureModeThreadLocal));
  }
  void launch_fwd(hipStream_t cs) {
    if (fexec) {
      CAPGEN_HIP(hipGraphLaunch(fexec, cs));
      return;
    }
    CAPGEN_HIP(hipGraphLaunch(fx[0], cs));
    dep(cs, es2, ev_ff);
    CAPGEN_HIP(hipGraphLaunch(fx[1], es2));
    hz::record(ev_fj, es2);
    CAPGEN_HIP(hipGraphLaunch(fx[2], cs));
    hz::wait(cs, ev_fj);
    CAPGEN_HIP(hipGraphLaunch(fx[3], cs));
  }
  bool have_fwd_graph() const { return fexec || fx[3]; }
  struct Key {
    const void *f, *p, *c;
    float* loss;
    int ft, B, N, T;
    bool drop;
    const void* idx;
    int nimg;
    bool operator==(const Key& o) const {
      return f == o.f && p == o.p && c == o.c && loss == o.loss && ft == o.ft && B == o.B && N == o.N && T == o.T &&
             drop == o.drop && idx == o.idx && nimg == o.nimg;
    }
  } gkey{}, fkey{};
  std::vector<std::array<int, 3>> tuned_shapes;
  bool tuned(int B, int N, int T) const {
    for (auto& t : tuned_shapes)
      if (t[0] == B && t[1] == N && t[2] == T) return true;
    return false;
  }
  // data parallel
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  float* count_host = nullptr;  // pinned: global count override
  hipEvent_t ev_count = nullptr;  // recorded after the copy of count_host (host writes wait for it)
  bool count_override = false;
  // sharded update (ZeRO-1, SURVEY §8(e) "later"): with world > 1 each bucket's gradients are
  // reduce-scattered, each rank runs Adam on its 1/world chunk only (its chunk of the moments is
  // the only one it keeps current), the updated f32 chunk is all-gathered in place and the bf16
  // shadow of the bucket re-cast locally.  Same bytes over xGMI as the all-reduce (RS + AG), 1/world
  // of the 1.67 GB Adam stream.  CAPGEN_ZERO=0: all-reduce + full Adam on every rank;
  // CAPGEN_ZERO=2: the sharded code path even at world 1 (RCCL test hook).
  int zero_mode = knob(Knob::Zero);
  int zemu_rank = 0, zemu_world = 1;  // capgen_dp_debug_shard: shard as rank r of w, no collectives
  // set by the sharded update: the Adam moments (resp. the gradient arena) are current in this rank's
  // chunks only until capgen_dp_sync_adam_state (resp. the next backward) -- the whole-arena getters
  // refuse them in between instead of returning stale data
  bool moments_sharded = false, grads_sharded = false;
  std::vector<std::array<int64_t, 2>> zbuckets;  // this step's bucket ranges, in issue order
  bool zbuckets_checked = false;
  int zworld() const {
    if (zemu_world > 1) return zemu_world;
    if (!comm || zero_mode == 0) return 1;
    return world > 1 || zero_mode == 2 ? world : 1;
  }
  int zrank() const { return zemu_world > 1 ? zemu_rank : rank; }
  bool zsharded() const { return zemu_world > 1 || (comm && (world > 1 ? zero_mode != 0 : zero_mode == 2)); }

  // ------------------------------------------------------------------------------------
  const void* W(int64_t off) const {
    return act == DType::BF16 ? (const void*)(shadow + off) : (const void*)(params + off);
  }
  const float* P(int64_t off) const { return params + off; }
  float* G(int64_t off) const { return grads + off; }
  float* GS(int64_t off) const { return gstripe + (off - L.enc_lng); }  // striped small-gradient slot
  void striped(LnBwd& lb) const { lb.stripes = NSTRIPE, lb.stripe_stride = n_small; }
  size_t es_() const { return dsize(act); }
  void* at(void* base, int64_t elems) const { return (char*)base + elems * es_(); }

  Drop mk_drop(float p, uint32_t site, bool on) const {
    Drop d{};
    if (!on || p <= 0.f) return d;
    d.seed_ptr = seed;
    d.site = site;
    d.thresh = drop_threshold(p);
    d.scale = 1.f / (1.f - p);
    return d;
  }
  // the f32 VALU attention backward reads the saved probabilities; the bf16 MFMA one recomputes
  bool keep_probs(const AttnGeom& g) const { return !(act == DType::BF16 && attention_mfma_ok(g)); }
  static uint32_t site(int dec, int layer, int kind) { return (uint32_t)((dec * 64 + layer) * 16 + kind); }

  // issue priority of a launch: kernels on the critical stream run their waves at s_setprio 3 so
  // that the weight-gradient / Adam waves of the side streams sharing their CUs yield the issue
  // slots to them (measured 2.779 / 2.788 vs 2.782 / 2.795 ms/step without, round 4)
  static constexpr bool prio_on = true;
  hipStream_t crit = nullptr;  // critical stream of the running call (es, or the caller's: direct)
  int prio(hipStream_t s) const { return prio_on && s == (crit ? crit : es) && es2 != s ? 1 : 0; }
  // direct steps: once the forward graph exists, train_step runs its
  // critical path on the CALLER's stream -- no caller -> engine -> caller event round trip per
  // step; es then waits for the step so the engine's host-side syncs on es still cover it
  // (measured: 3.165 vs 3.170 ms/step, within noise -- the step-boundary gap is the Adam tail)
  // fused classifier + cross entropy in the bf16 path (CAPGEN_FUSED_CE=0: logits in f32 + ce_kernel)
  bool fused_ce_on = knob(Knob::FusedCe) != 0;
  bool need_logits = false;  // the next forward must materialise the f32 logits (SCST sampling)
  bool fused_ce() const { return fused_ce_on && !need_logits && act == DType::BF16 && L_().V % 4 == 0; }
  // train step without a collective or FocalLoss: the CE gradient scale 1/count comes from the caption
  // prep (the count is known there), so the loss finalisation (the mean of the loss rows) leaves the
  // critical stream: the step's forward skips it and its backward issues it on es2 after the first
  // fork (pending_loss).  With a count all-reduce or FocalLoss the scale needs the finalisation first.
  bool loss_deferrable() const { return !comm && !count_override && !cfg.focal_loss && defer_loss_on; }
  bool defer_loss_on = knob(Knob::DeferLoss) != 0;
  int front_join = knob(Knob::FrontJoin);  // encoder block before which the forward joins the decoder front
  float* pending_loss = nullptr;  // set by train_step: the backward finalises the loss into it on es2
  static constexpr bool direct_on = true;

  // diagnostic in-kernel timestamps (capgen_debug_stamps): every GEMM / LayerNorm / attention
  // launch of a step gets a slot of the ring (forward slots first: a captured forward graph keeps
  // its slots, the backward re-numbers from where the forward ended); names for the report
  bool stamp_on = false;
  uint64_t* stamp_ring = nullptr;
  static constexpr int kStampSlots = 4096;
  int stamp_next = 0, stamp_fwd_end = 0, stamp_max = 0;
  std::vector<std::string> stamp_names;
  uint64_t* stamp(hipStream_t s, const std::string& what) {
    if (!stamp_on || !stamp_ring || stamp_next >= kStampSlots) return nullptr;
    const int i = stamp_next++;
    stamp_max = std::max(stamp_max, stamp_next);
    if ((int)stamp_names.size() <= i) stamp_names.resize(i + 1);
    stamp_names[i] = std::string(s == ec && ec != es2 ? "bucket " : s == es2 && es2 != (crit ? crit : es) ? "side " : "crit ") + what;
    return stamp_ring + (size_t)i * 16;
  }
  static std::string dims(int M, int N, int K) {
    return std::to_string(M) + "x" + std::to_string(N) + "x" + std::to_string(K);
  }

  // the row / attention kernels with the launch's issue priority (prio above)
  void lnf(LnFwd l, hipStream_t s) {
    l.prio = prio(s);
    if (stamp_on) l.stamp = stamp(s, "ln_fwd " + std::to_string(l.M));
    layernorm_fwd(l, act, s);
  }
  void lnb(LnBwd l, hipStream_t s) {
    l.prio = prio(s);
    if (stamp_on) l.stamp = stamp(s, "ln_bwd " + std::to_string(l.M));
    layernorm_bwd(l, act, s);
  }
  void attf(AttnGeom g, void* o, float* probs, DType t, hipStream_t s) {
    g.prio = prio(s);
    if (stamp_on) g.stamp = stamp(s, "attn_fwd " + std::to_string(g.Lq) + "x" + std::to_string(g.Lk));
    attention_fwd(g, o, probs, t, s);
  }
  void attb(AttnGeom g, const float* probs, const void* dout, void* dq, void* dk, void* dv, DType t,
            hipStream_t s) {
    g.prio = prio(s);
    if (stamp_on) g.stamp = stamp(s, "attn_bwd " + std::to_string(g.Lq) + "x" + std::to_string(g.Lk));
    attention_bwd(g, probs, dout, dq, dk, dv, t, s);
  }

  // The self-attention front of a block (modules.py:67-76 + 16-27): qkv = X . Wqkv^T, then the
  // attention of g over it into att.  bf16 with head size 64 and d = 512: ONE fused launch
  // (qkv_attn.hip: projection straight into the attention's LDS images; qkv still written for the
  // backward).  Otherwise (f32 parity mode, other geometries, CAPGEN_FUSED_QKV=0) the GEMM and the
  // attention launch.
  bool fused_qkv_on = knob(Knob::FusedQkv) != 0;
  void self_attention(const void* X, int64_t wqkv, int M, int d, const AttnGeom& g, void* qkv, void* att, float* probs,
                      hipStream_t s) {
    if (fused_qkv_on && act == DType::BF16 && !keep_probs(g)) {
      QkvAttn qa;
      qa.g = g, qa.g.prio = prio(s);
      qa.X = reinterpret_cast<const bf16*>(X), qa.ldx = d, qa.W = WT(wqkv);
      qa.d = d, qa.qkv = reinterpret_cast<bf16*>(qkv), qa.ldqkv = 3 * d, qa.o = reinterpret_cast<bf16*>(att);
      if (qkv_attn_ok(qa)) {
        if (stamp_on) qa.g.stamp = stamp(s, "qkv_attn " + std::to_string(g.Lq) + "x" + std::to_string(g.Lk));
        qkv_attn_fwd(qa, s);
        return;
      }
    }
    linear(X, d, wqkv, d, qkv, 3 * d, act, M, 3 * d, d, nullptr, 0, s);
    attf(g, att, probs, act, s);
  }

  // The cross-attention of a decoder block (modules.py:195-197): q = D1 . Wq^T then attention over
  // the precomputed cross K/V.  q_done: q already projected (else bf16: the fused launch projects it
  // straight into the attention's LDS image, qkv_attn.hip cross mode).
  bool cross_fusable(int Lq) const {
    return fused_qkv_on && act == DType::BF16 && wtile && L.dd == 512 && L.Hd * 64 == L.dd && Lq >= 1 && Lq <= 64;
  }
  void cross_attention(const AttnGeom& c, const void* D1, int64_t wq, int d, void* qc, void* attc, float* probs,
                       bool q_done, hipStream_t s) {
    if (!q_done) {
      QkvAttn qa;
      qa.g = c, qa.g.prio = prio(s), qa.cross = 1;
      qa.X = reinterpret_cast<const bf16*>(D1), qa.ldx = d, qa.W = WT(wq);
      qa.d = d, qa.qkv = reinterpret_cast<bf16*>(qc), qa.ldqkv = d, qa.o = reinterpret_cast<bf16*>(attc);
      require(!probs && qkv_attn_ok(qa), "internal: cross-attention geometry the fused launch does not take");
      if (stamp_on) qa.g.stamp = stamp(s, "qkv_attn cross " + std::to_string(c.Lq) + "x" + std::to_string(c.Lk));
      qkv_attn_fwd(qa, s);
      return;
    }
    attf(c, attc, probs, act, s);
  }

  // C[M,N] = A[M,K] . W[N,K]^T  (nn.Linear)
  // bt: the weight's fragment pieces (DT), read by the register-B GEMM where it takes the shape
  void linear(const void* X, int64_t ldx, int64_t woff, int64_t ldw, void* C, int64_t ldc, DType tout, int M,
              int N, int K, const float* bias, int relu, hipStream_t s, const void* bt = nullptr) {
    GemmArgs ga;
    ga.M = M, ga.N = N, ga.K = K, ga.A = X, ga.lda = ldx, ga.B = W(woff), ga.ldb = ldw, ga.C = C, ga.ldc = ldc;
    ga.bt = bt;
    ga.bias = bias;
    ga.relu = relu;
    ga.prio = prio(s);
    if (stamp_on) ga.stamp = stamp(s, "gemm fwd " + dims(M, N, K));
    gemm(ga, act, tout, false, false, s);
  }
  // C = X . W^T into ln.a, then y = LayerNorm(drop(C + bias) + res (+ pe)) (modules.py:86-90).
  // (Fusing the LayerNorm into the GEMM -- a row-block finisher reloading the rows write-through
  // -- was measured slower than this separate launch: DESIGN.md section 6.)
  void linear_ln(const void* X, int64_t ldx, int64_t woff, int64_t ldw, int M, int N, int K, const LnFwd& ln,
                 hipStream_t s) {
    linear(X, ldx, woff, ldw, const_cast<void*>(ln.a), N, act, M, N, K, nullptr, 0, s);
    lnf(ln, s);
  }
  // a LayerNorm backward descriptor (striped accumulators); b_off < 0: no producing-Linear bias
  LnBwd lnb_desc(int M, int d, const void* dy, const void* v, const float* mean, const float* rstd, int64_t lng,
                 int64_t lnb, int64_t b_off, RowMask mask, Drop drop, void* d_res, void* d_a) const {
    LnBwd lb;
    lb.M = M, lb.d = d, lb.dy = dy, lb.v = v, lb.mean = mean, lb.rstd = rstd, lb.gamma = P(lng), lb.mask = mask;
    lb.drop = drop, lb.d_res = d_res, lb.d_a = d_a, lb.dgamma = GS(lng), lb.dbeta = GS(lnb);
    lb.dbias = b_off >= 0 ? GS(b_off) : nullptr;
    striped(lb);
    return lb;
  }

  // dX[M,K] (+)= alpha * dY[M,N] . W[N,K]
  void linear_dx(const void* dY, int64_t ldy, int64_t woff, int64_t ldw, void* dX, int64_t ldx, int M, int N, int K,
                 int beta, const void* relu_aux, const float* alpha_ptr, hipStream_t s, float* colsum = nullptr) {
    GemmArgs ga;
    ga.colsum = colsum;
    ga.colsum_stripes = NSTRIPE, ga.colsum_stride = n_small;  // colsum always targets gstripe
    ga.M = M, ga.N = K, ga.K = N, ga.A = dY, ga.lda = ldy, ga.B = W(woff), ga.ldb = ldw, ga.C = dX, ga.ldc = ldx;
    ga.beta = beta;
    ga.aux = relu_aux;
    ga.ldaux = ldx;
    ga.alpha_ptr = alpha_ptr;
    ga.prio = prio(s);
    if (stamp_on) ga.stamp = stamp(s, "gemm dX " + dims(M, K, N));
    gemm(ga, act, act, false, true, s);
  }
  // dW[N,K] = alpha * dY[M,N]^T . X[M,K]   (f32, overwrites)
  void linear_dw(const void* dY, int64_t ldy, const void* X, int64_t ldx, int64_t goff, int64_t ldg, int M, int N,
                 int K, const float* alpha_ptr, hipStream_t s) {
    GemmArgs ga;
    ga.M = N, ga.N = K, ga.K = M, ga.A = dY, ga.lda = ldy, ga.B = X, ga.ldb = ldx, ga.C = G(goff), ga.ldc = ldg;
    ga.alpha_ptr = alpha_ptr;
    ga.prio = prio(s);
    if (stamp_on) ga.stamp = stamp(s, "gemm dW " + dims(N, K, M));
    gemm(ga, act, DType::F32, true, true, s);
  }

  // ------------------------------------------------------------------------------------
  void plan_acts(Planner& p, int B, int N, int T) {
    const int64_t Me = (int64_t)B * N, L = T - 1, Md = (int64_t)B * L, d = L_().d, dd = L_().dd;
    const int64_t Mx = std::max(Me, Md);
    const size_t e = es_();
    auto T_ = [&](void*& ptr, int64_t n) { ptr = p.raw(n * e); };
    T_(a.Aenc, Me * L_().Kp);
    p.take(a.valid, Me);
    T_(a.ev0, Me * d);
    p.take(a.em0, Me);
    p.take(a.er0, Me);
    a.X.resize(L_().Le + 1);
    for (auto& x : a.X) T_(x, Me * d);
    a.enc.resize(L_().Le);
    for (auto& l : a.enc) {
      T_(l.qkv, Me * 3 * d);
      p.take(l.P, (size_t)B * L_().He * N * N);
      T_(l.att, Me * d);
      T_(l.v1, Me * d);
      p.take(l.m1, Me);
      p.take(l.r1, Me);
      T_(l.Y, Me * d);
      T_(l.H, Me * L_().fe);
      T_(l.v2, Me * d);
      p.take(l.m2, Me);
      p.take(l.r2, Me);
    }
    T_(a.KV, Me * L_().Ld * 2 * dd);
    p.take(a.ids, Md);
    p.take(a.tgt, Md);
    p.take(a.count, 4);
    T_(a.E, Md * L_().dwe);
    T_(a.dv0, Md * dd);
    T_(a.tmpf, Md * dd);
    p.take(a.dm0, Md);
    p.take(a.dr0, Md);
    a.D.resize(L_().Ld + 1);
    for (auto& x : a.D) T_(x, Md * dd);
    a.dec.resize(L_().Ld);
    for (auto& l : a.dec) {
      T_(l.qkv, Md * 3 * dd);
      p.take(l.Ps, (size_t)B * L_().Hd * L * L);
      T_(l.atts, Md * dd);
      T_(l.vs, Md * dd);
      p.take(l.ms, Md);
      p.take(l.rs, Md);
      T_(l.D1, Md * dd);
      T_(l.qc, Md * dd);
      p.take(l.Pc, (size_t)B * L_().Hd * L * N);
      T_(l.attc, Md * dd);
      T_(l.vc, Md * dd);
      p.take(l.mc, Md);
      p.take(l.rc, Md);
      T_(l.D2, Md * dd);
      T_(l.H, Md * L_().fd);
      T_(l.vf, Md * dd);
      p.take(l.mf, Md);
      p.take(l.rf, Md);
    }
    p.take(a.logits, Md * L_().V);
    T_(a.dlogits, Md * L_().V);
    a.ce_stats = reinterpret_cast<float2*>(p.raw((size_t)Md * ((L_().V + 15) / 16) * sizeof(float2)));
    p.take(a.ce_tl, Md);
    p.take(a.loss_row, Md);
    p.take(a.grad_scale, 4);
    p.take(a.loss, 4);
    p.take(a.loss_ce, 4);
    T_(a.gEnc, Me * d);
    p.take(a.rl_sample, Md);
    p.take(a.rl_lse, Md);
    p.take(a.rl_logp, Md);
    p.take(a.rl_ent, Md);
    p.take(a.rl_ent_img, B);
    p.take(a.rl_score, B);
    p.take(a.rl_scal, 8);
    const int64_t dmax = std::max<int64_t>(std::max(d, dd), L_().dwe);
    T_(a.tmp, Mx * dmax);
    T_(a.gOut, Mx * dmax);
    T_(a.gRes, Mx * dmax);
    T_(a.gKV, Me * L_().Ld * 2 * dd);
    T_(a.gE, Md * L_().dwe);
    T_(a.gAe, Me * d);
    T_(a.gAd, Md * dd);
    a.genc.resize(L_().Le);
    for (auto& gb : a.genc) {
      T_(gb.gAf, Me * d);
      T_(gb.gH, Me * L_().fe);
      T_(gb.gA1, Me * d);
      T_(gb.gATT1, Me * d);
      T_(gb.gQKV, Me * 3 * d);
      gb.gA2 = gb.gATT2 = gb.gQc = nullptr;
    }
    if (L_().has_img) {  // sized 0 otherwise (the planner still hands out aligned pointers)
      const int64_t M2 = 2 * Me;
      T_(a.siY, Me * d);
      T_(a.siEp, Me * d);
      T_(a.siX2, M2 * d);
      T_(a.siZ, M2 * d);
      T_(a.siV, Me * d);
      T_(a.siG0, M2 * d);
      T_(a.siG1, M2 * d);
      T_(a.siGY, Me * d);
      T_(a.siGEp, Me * d);
      p.take(a.siValid, M2);
      p.take(a.siM, Me);
      p.take(a.siR, Me);
      auto& l = a.si;
      T_(l.qkv, M2 * 3 * d);
      p.take(l.P, (size_t)Me * L_().He * 4);
      T_(l.att, M2 * d);
      T_(l.v1, M2 * d);
      p.take(l.m1, M2);
      p.take(l.r1, M2);
      T_(l.Y, M2 * d);
      T_(l.H, M2 * L_().fe);
      T_(l.v2, M2 * d);
      p.take(l.m2, M2);
      p.take(l.r2, M2);
      auto& gb = a.gsi;
      T_(gb.gAf, M2 * d);
      T_(gb.gH, M2 * L_().fe);
      T_(gb.gA1, M2 * d);
      T_(gb.gATT1, M2 * d);
      T_(gb.gQKV, M2 * 3 * d);
      gb.gA2 = gb.gATT2 = gb.gQc = nullptr;
    }
    if (L_().has_mf) {
      T_(a.mfU, Md * dd);
      T_(a.mfH, Md * L_().fd);
      T_(a.mfV, Md * dd);
      T_(a.mfOut, Md * dd);
      T_(a.mfGA, Md * dd);
      T_(a.mfGH, Md * L_().fd);
      T_(a.mfGU, Md * dd);
      p.take(a.mfM, Md);
      p.take(a.mfR, Md);
    }
    a.gdec.resize(L_().Ld);
    for (auto& gb : a.gdec) {
      T_(gb.gAf, Md * dd);
      T_(gb.gH, Md * L_().fd);
      T_(gb.gA1, Md * dd);
      T_(gb.gATT1, Md * dd);
      T_(gb.gQKV, Md * 3 * dd);
      T_(gb.gA2, Md * dd);
      T_(gb.gATT2, Md * dd);
      T_(gb.gQc, Md * dd);
    }
  }
  const Layout& L_() const { return L; }

  void ensure_acts(int B, int N, int T) {
    if (ws && B <= a.B && N <= a.N && T <= a.T) return;
    int nB = std::max(B, a.B), nN = std::max(N, a.N), nT = std::max(T, a.T);
    if (ws) {
      hz::host_sync(es);
      CAPGEN_HIP(hipFree(ws));
      ws = nullptr;
      drop_graph();
    }
    Planner p;
    plan_acts(p, nB, nN, nT);
    CAPGEN_HIP(hipMalloc(&ws, p.used));
    Planner q;
    q.base = (char*)ws;
    plan_acts(q, nB, nN, nT);
    a.B = nB, a.N = nN, a.T = nT;
  }

  void drop_graph() {
    if (gexec) {
      (void)hipGraphExecDestroy(gexec);
      gexec = nullptr;
    }
    for (auto& x : fx)
      if (x) (void)hipGraphExecDestroy(x), x = nullptr;
    if (fexec) {
      (void)hipGraphExecDestroy(fexec);
      fexec = nullptr;
    }
    drop_gen_graph();
  }
  void drop_gen_graph() {
    for (auto& e : gen_graphs) (void)hipGraphExecDestroy(e.second);
    gen_graphs.clear();
    gen_seen.clear();
  }

  // Decoding as one replayed hipGraph: the first call with a given
  // (kind, inputs, shape) runs eagerly (autotunes the GEMMs, sizes the workspaces), the second
  // captures the whole encode + T-1 decode steps on the engine stream, later ones replay it.
  // Outputs are staged in the workspace (g.out_*) and copied to the caller's buffers after
  // the launch, so a new output tensor per call does not defeat the replay.
  // decode scoring: false = Softmax, probabilities accumulated over beams (Transformer,
  // model.py:124-128,183); true = LogSoftmax, log-probabilities (PolicyNetwork, model_RL.py:72,182)
  bool decode_logsm = false;
  struct GenKey {
    int kind;  // 0 greedy, 1 greedy + attention, 2 beam (+ 8: log-softmax scoring)
    const void *f, *p;
    int ft, B, N, k;
    bool operator==(const GenKey& o) const {
      return kind == o.kind && f == o.f && p == o.p && ft == o.ft && B == o.B && N == o.N && k == o.k;
    }
  };
  // off by default: measured slower than eager issue on MI355X / ROCm 7 (C4 B=256: beam 5
  // 22.6 vs 21.9 ms, greedy 12.4 vs 11.6 ms, tools/bench_generate.py); CAPGEN_GEN_GRAPH=1 enables
  bool gen_graph_on = knob(Knob::GenGraph) == 1;
  static constexpr size_t kGenGraphs = 8;  // cached decode graphs (oldest evicted)
  std::vector<std::pair<GenKey, hipGraphExec_t>> gen_graphs;
  std::vector<GenKey> gen_seen;  // keys run eagerly once (next call captures)
  template <class F>
  void gen_run(const GenKey& k, F&& body, hipStream_t s) {
    if (!gen_graph_on) return body();
    for (auto& e : gen_graphs)
      if (e.first == k) {
        CAPGEN_HIP(hipGraphLaunch(e.second, s));
        return;
      }
    if (std::find(gen_seen.begin(), gen_seen.end(), k) == gen_seen.end()) {  // first sighting: eager
      body();
      gen_seen.push_back(k);
      if (gen_seen.size() > kGenGraphs) gen_seen.erase(gen_seen.begin());
      return;
    }
    const GenWS saved = g;  // beam's host-side ping-pong swaps are replayed from this state
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    CAPGEN_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    try {
      body();
    } catch (...) {
      (void)hipStreamEndCapture(s, &graph);
      if (graph) (void)hipGraphDestroy(graph);
      g = saved;
      throw;
    }
    CAPGEN_HIP(hipStreamEndCapture(s, &graph));
    g = saved;
    CAPGEN_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    CAPGEN_HIP(hipGraphDestroy(graph));
    if (gen_graphs.size() >= kGenGraphs) {
      (void)hipGraphExecDestroy(gen_graphs.front().second);
      gen_graphs.erase(gen_graphs.begin());
    }
    gen_graphs.emplace_back(k, exec);
    CAPGEN_HIP(hipGraphLaunch(exec, s));
  }

  // ------------------------------------------------------------------------------------
  // one EncoderBlock (modules.py:146-157) over B sequences of N rows: X -> Xout.  valid != null:
  // key-pad OR causal self-attention mask and the non-pad multiply (model.py:312-328).
  void enc_layer_fwd(const EncLayerOff& w, EncAct& A, const void* X, void* Xout, int B, int N, const uint8_t* valid,
                     int layer, bool drop_on, hipStream_t s) {
    const int Me = B * N, d = L.d, He = L.He, dke = d / He;
    const float p = cfg.dropout, pa = cfg.attention_dropout;
    AttnGeom g;
    g.B = B, g.H = He, g.Lq = N, g.Lk = N, g.dk = dke;
    g.q = A.qkv, g.q_ld = 3 * d, g.q_bs = (int64_t)N * 3 * d;
    g.k = at(A.qkv, d), g.k_ld = 3 * d, g.k_bs = (int64_t)N * 3 * d;
    g.v = at(A.qkv, 2 * d), g.v_ld = 3 * d, g.v_bs = (int64_t)N * 3 * d;
    g.o_ld = d, g.o_bs = (int64_t)N * d;
    if (valid) g.key_valid = valid, g.kv_bs = N, g.causal = 1;
    g.temperature = std::sqrt((float)dke);
    g.drop = mk_drop(pa, site(0, layer, 0), drop_on);
    self_attention(X, w.Wqkv, Me, d, g, A.qkv, A.att, keep_probs(g) ? A.P : nullptr, s);
    LnFwd l1;
    l1.M = Me, l1.d = d, l1.a = a.tmp, l1.drop = mk_drop(p, site(0, layer, 1), drop_on), l1.res = X;
    l1.gamma = P(w.ln1g), l1.beta = P(w.ln1b), l1.y = A.Y, l1.v_save = A.v1, l1.mean = A.m1, l1.rstd = A.r1;
    linear_ln(A.att, d, w.Wo, d, Me, d, d, l1, s);
    linear(A.Y, d, w.W1, d, A.H, L.fe, act, Me, L.fe, d, P(w.b1), 1, s);
    LnFwd l2;
    l2.M = Me, l2.d = d, l2.a = a.tmp, l2.a_bias = P(w.b2), l2.drop = mk_drop(p, site(0, layer, 2), drop_on);
    l2.res = A.Y, l2.gamma = P(w.ln2g), l2.beta = P(w.ln2b), l2.mask.valid = valid;
    l2.y = Xout, l2.v_save = A.v2, l2.mean = A.m2, l2.rstd = A.r2;
    linear_ln(A.H, L.fe, w.W2, L.fe, Me, d, L.fe, l2, s);
  }
  static constexpr int kImgLayer = 63;  // dropout-site layer index of encoder.image_encoder

  // split_image_objects (model.py:258-292, then the shared norm :294): a.Aenc -> a.X[0]
  void image_objects_fwd(int B, int N, bool drop_on, hipStream_t s) {
    const int Me = B * N, d = L.d;
    // LN([feats | pos] . W^T) per token; the pair rows only repeat rows, so embed each region once
    LnFwd ln;
    ln.M = Me, ln.d = d, ln.a = a.tmp, ln.gamma = P(L.enc_lng), ln.beta = P(L.enc_lnb);
    ln.y = a.siY, ln.v_save = a.ev0, ln.mean = a.em0, ln.rstd = a.er0;
    linear_ln(a.Aenc, L.Kp, L.enc_emb_W, L.Kp, Me, d, L.Kp, ln, s);
    // the position embedding alone (added to the region token after the image block): the
    // position columns [F, Kp) of the packed input and weight (zero beyond F + P)
    linear(at(a.Aenc, L.F), L.Kp, L.enc_emb_W + L.F, L.Kp, a.siEp, d, act, Me, d, L.Kp - L.F, nullptr, 0, s);
    pair_gather(a.siY, a.valid, B, N, d, a.siX2, a.siValid, act, s);
    enc_layer_fwd(L.img, a.si, a.siX2, a.siZ, Me, 2, a.siValid, kImgLayer, drop_on, s);
    pair_take_add(a.siZ, a.siEp, Me, d, a.tmp, act, s);
    LnFwd l2;
    l2.M = Me, l2.d = d, l2.a = a.tmp, l2.gamma = P(L.enc_lng), l2.beta = P(L.enc_lnb);
    l2.y = a.X[0], l2.v_save = a.siV, l2.mean = a.siM, l2.rstd = a.siR;
    lnf(l2, s);
  }
  static constexpr int kMfLayer = 62;  // dropout-site layer index of the decoder's move-first FFN

  // move_first_image_feature (model.py:451-457): y = LN(x + drop(W2 relu(W1 (x + enc[:, 0]) + b1) + b2))
  // over the M decoder rows in x (row r -> image r / rows_per_img, or r % bmod)
  void move_first_fwd(const void* x, const void* enc, int M, int rows_per_img, int bmod, int N, void* U, void* H,
                      void* tmp, void* y, void* v_save, float* mean, float* rstd, bool drop_on, hipStream_t s) {
    const int dd = L.dd;
    add_first_region(x, enc, M, rows_per_img, bmod, N, dd, U, act, s);
    linear(U, dd, L.mf_W1, dd, H, L.fd, act, M, L.fd, dd, P(L.mf_b1), 1, s);
    LnFwd ln;
    ln.M = M, ln.d = dd, ln.a = tmp, ln.a_bias = P(L.mf_b2), ln.drop = mk_drop(cfg.dropout, site(1, kMfLayer, 0), drop_on);
    ln.res = x, ln.gamma = P(L.mf_lng), ln.beta = P(L.mf_lnb), ln.y = y, ln.v_save = v_save, ln.mean = mean;
    ln.rstd = rstd;
    linear_ln(H, L.fd, L.mf_W2, L.fd, M, dd, L.fd, ln, s);
  }
  // the decoder output the classifier reads
  void* dec_out() const { return L.has_mf ? a.mfOut : a.D[L.Ld]; }

  // ------------------------------------------------------------------------------------
  // forward (model.py:79-98).  Always keeps the activations needed by backward.
  void forward(const void* feats, DType ft, const float* pos, const int32_t* caps, int B, int N, int T,
               float* loss_out, bool drop_on, hipStream_t s, bool defer_loss = false) {
    const bool defer = defer_loss && loss_deferrable();
    require(B >= 1 && N >= 1 && T >= 2, "forward: need B>=1, N>=1, T>=2");
    require(N <= 64 && T - 1 <= L.maxlen - 1, "forward: N must be <= 64 and T <= max_length");
    const int Lq = T - 1, Me = B * N, Md = B * Lq, d = L.d, dd = L.dd;
    const int He = L.He, Hd = L.Hd, dke = d / He, dkd = dd / Hd;
    fB = B, fN = N, fT = T, fwd_drop = drop_on;
    stamp_next = 0;
    const float p = cfg.dropout, pa = cfg.attention_dropout;

    // (+ the dropout seed advance when dropout is on: the pack kernel does not read the seed, every
    // dropout site of this forward runs after this launch)
    pack_encoder_input(feats, ft, pos, Me, L.F, L.P, L.Kp, a.Aenc, act, a.valid, s, in_idx, N, in_n_img,
                       drop_on ? seed : nullptr);
    // caption ids / targets / count: with the decoder front on es2 (and no count all-reduce, which
    // stays on the critical stream) the prep runs there too, first thing of the front
    const bool caps_front = overlap_front && es2 != s && !comm;
    if (!caps_front) prepare_captions(caps, B, T, cfg.pad_idx, a.ids, a.tgt, a.count, s, nullptr, defer ? a.grad_scale : nullptr);
    if (comm) {
      if (count_override) {
        if (hz::active()) hz::op(s, "count_copy", {hz::wr(a.count, 4)});
        CAPGEN_HIP(hipMemcpyAsync(a.count, count_host, sizeof(float), hipMemcpyHostToDevice, s));
        hz::record(ev_count, s);  // capgen_dp_set_global_count waits for this copy
      }
      else {
        nccl_op(s, "allreduce(count)", a.count, 4);
        NCCL_CHECK(ncclAllReduce(a.count, a.count, 1, ncclFloat, ncclSum, comm, s));
      }
    }

    // ---- decoder front (model.py:432-436 and block 0's self-attention half + cross query,
    // modules.py:185-197): depends on the captions only, so with overlap_front it runs on es2
    // beside the whole encoder and joins before block 0's cross attention
    RowMask dmask{};
    dmask.ids = a.ids, dmask.pad_idx = cfg.pad_idx;
    const bool front = overlap_front && es2 != s;
    auto dec_embed = [&](void* tmp, hipStream_t fs) {
      embedding_gather(P(L.emb), a.ids, 1, Md, L.dwe, a.E, act, fs, L.V);
      LnFwd ln;
      ln.M = Md, ln.d = dd, ln.a = tmp, ln.pe = pe, ln.pe_L = Lq, ln.gamma = P(L.dec_lng), ln.beta = P(L.dec_lnb);
      ln.y = a.D[0], ln.v_save = a.dv0, ln.mean = a.dm0, ln.rstd = a.dr0;
      linear_ln(a.E, L.dwe, L.Wel, L.dwe, Md, dd, L.dwe, ln, fs);
    };
    // self attention: key-pad(ids) OR causal (model.py:421-430), then the cross-attention query
    // q_proj: also the cross-attention query projection (else the fused cross-attention launch does it)
    auto dec_self_half = [&](int l, void* tmp, hipStream_t fs, bool q_proj) {
      const auto& w = L.dec[l];
      auto& A = a.dec[l];
      AttnGeom g;
      g.B = B, g.H = Hd, g.Lq = Lq, g.Lk = Lq, g.dk = dkd;
      g.q = A.qkv, g.q_ld = 3 * dd, g.q_bs = (int64_t)Lq * 3 * dd;
      g.k = at(A.qkv, dd), g.k_ld = 3 * dd, g.k_bs = (int64_t)Lq * 3 * dd;
      g.v = at(A.qkv, 2 * dd), g.v_ld = 3 * dd, g.v_bs = (int64_t)Lq * 3 * dd;
      g.o_ld = dd, g.o_bs = (int64_t)Lq * dd;
      g.key_ids = a.ids, g.kid_bs = Lq, g.pad_idx = cfg.pad_idx, g.causal = 1;
      g.temperature = std::sqrt((float)dkd);
      g.drop = mk_drop(pa, site(1, l, 3), drop_on);
      self_attention(a.D[l], w.Wqkv, Md, dd, g, A.qkv, A.atts, keep_probs(g) ? A.Ps : nullptr, fs);
      LnFwd l1;
      l1.M = Md, l1.d = dd, l1.a = tmp, l1.drop = mk_drop(p, site(1, l, 4), drop_on), l1.res = a.D[l];
      l1.gamma = P(w.lsg), l1.beta = P(w.lsb), l1.y = A.D1, l1.v_save = A.vs, l1.mean = A.ms, l1.rstd = A.rs;
      linear_ln(A.atts, dd, w.Wo_s, dd, Md, dd, dd, l1, fs);
      if (q_proj) linear(A.D1, dd, w.Wq_c, dd, A.qc, dd, act, Md, dd, dd, nullptr, 0, fs);
    };
    if (front) {
      if (cap_split) cap_cut(s, 0, es2);
      else dep(s, es2, ev_ff);
      if (caps_front) prepare_captions(caps, B, T, cfg.pad_idx, a.ids, a.tgt, a.count, es2, nullptr, defer ? a.grad_scale : nullptr);
      dec_embed(a.tmpf, es2);
      dec_self_half(0, a.tmpf, es2, true);
      if (cap_split) cap_cut(es2, 1, s);
      else hz::record(ev_fj, es2);
    }

    // ---- encoder (model.py:294-332) ----
    if (L.has_img) {
      image_objects_fwd(B, N, drop_on, s);
    } else {
      LnFwd ln;
      ln.M = Me, ln.d = d, ln.a = a.tmp, ln.gamma = P(L.enc_lng), ln.beta = P(L.enc_lnb);
      ln.y = a.X[0], ln.v_save = a.ev0, ln.mean = a.em0, ln.rstd = a.er0;
      linear_ln(a.Aenc, L.Kp, L.enc_emb_W, L.Kp, Me, d, L.Kp, ln, s);
    }
    // where the critical stream joins the decoder front (eager / single graph): before encoder block
    // front_join (Le + 1: before the decoder, its first reader)
    const int fj = std::max(0, std::min(front_join, L.Le + 1));
    for (int l = 0; l < L.Le; ++l) {
      if (front && !cap_split && l == fj) hz::wait(s, ev_fj);
      enc_layer_fwd(L.enc[l], a.enc[l], a.X[l], a.X[l + 1], B, N, cfg.encode_mask ? a.valid : nullptr, l, drop_on, s);
    }
    if (front && !cap_split && fj == L.Le) hz::wait(s, ev_fj);
    // cross-attention K/V of every decoder block in one GEMM over the encoder output
    linear(a.X[L.Le], d, L.Wkv_all, d, a.KV, (int64_t)L.Ld * 2 * dd, act, Me, L.Ld * 2 * dd, d, nullptr, 0, s);

    // ---- decoder (model.py:419-459) ----
    if (front && cap_split) cap_cut(s, 2, s);
    else if (front && fj > L.Le) hz::wait(s, ev_fj);
    else if (!front) dec_embed(a.tmp, s);
    const int64_t kvld = (int64_t)L.Ld * 2 * dd;
    for (int l = 0; l < L.Ld; ++l) {
      const auto& w = L.dec[l];
      auto& A = a.dec[l];
      const bool q_done = front && l == 0;  // block 0's query was projected on es2 with the front
      if (!q_done) dec_self_half(l, a.tmp, s, !cross_fusable(Lq));
      // cross attention over the encoder output, context mask = region key-pad (model.py:82)
      AttnGeom c;
      c.B = B, c.H = Hd, c.Lq = Lq, c.Lk = N, c.dk = dkd;
      c.q = A.qc, c.q_ld = dd, c.q_bs = (int64_t)Lq * dd;
      c.k = at(a.KV, (int64_t)l * 2 * dd), c.k_ld = kvld, c.k_bs = (int64_t)N * kvld;
      c.v = at(a.KV, (int64_t)l * 2 * dd + dd), c.v_ld = kvld, c.v_bs = (int64_t)N * kvld;
      c.o_ld = dd, c.o_bs = (int64_t)Lq * dd;
      c.key_valid = a.valid, c.kv_bs = N;
      c.temperature = std::sqrt((float)dkd);
      c.drop = mk_drop(pa, site(1, l, 5), drop_on);
      cross_attention(c, A.D1, w.Wq_c, dd, A.qc, A.attc, keep_probs(c) ? A.Pc : nullptr, q_done || !cross_fusable(Lq), s);
      LnFwd l2;
      l2.M = Md, l2.d = dd, l2.a = a.tmp, l2.drop = mk_drop(p, site(1, l, 6), drop_on), l2.res = A.D1;
      l2.gamma = P(w.lcg), l2.beta = P(w.lcb), l2.y = A.D2, l2.v_save = A.vc, l2.mean = A.mc, l2.rstd = A.rc;
      linear_ln(A.attc, dd, w.Wo_c, dd, Md, dd, dd, l2, s);
      // FFN, then x non_pad (modules.py:201-204)
      linear(A.D2, dd, w.W1, dd, A.H, L.fd, act, Md, L.fd, dd, P(w.b1), 1, s);
      LnFwd l3;
      l3.M = Md, l3.d = dd, l3.a = a.tmp, l3.a_bias = P(w.b2), l3.drop = mk_drop(p, site(1, l, 7), drop_on);
      l3.res = A.D2, l3.gamma = P(w.lfg), l3.beta = P(w.lfb), l3.mask = dmask;
      l3.y = a.D[l + 1], l3.v_save = A.vf, l3.mean = A.mf, l3.rstd = A.rf;
      linear_ln(A.H, L.fd, w.W2, L.fd, Md, dd, L.fd, l3, s);
    }
    if (L.has_mf)
      move_first_fwd(a.D[L.Ld], a.X[L.Le], Md, Lq, 0, N, a.mfU, a.mfH, a.tmp, a.mfOut, a.mfV, a.mfM, a.mfR, drop_on, s);
    // ---- classifier + CE (model.py:93-96) ----
    if (fused_ce()) {
      // the logits are never written: the GEMM epilogue leaves exp(v - slab max) + slab stats,
      // ce_finish turns them into the loss rows and softmax - onehot (model.py:93-96)
      GemmArgs ga;
      ga.M = Md, ga.N = L.V, ga.K = dd, ga.A = dec_out(), ga.lda = dd, ga.B = W(L.Wc), ga.ldb = dd;
      ga.C = a.dlogits, ga.ldc = L.V, ga.bias = P(L.bc), ga.prio = prio(s);
      ga.ce_stats = a.ce_stats, ga.ce_ld = (L.V + 15) / 16, ga.ce_tgt = a.tgt, ga.ce_tlogit = a.ce_tl;
      if (stamp_on) ga.stamp = stamp(s, "gemm classifier+CE " + dims(Md, L.V, dd));
      gemm(ga, act, act, false, false, s);
      ce_finish(a.ce_stats, (L.V + 15) / 16, a.ce_tl, a.tgt, Md, L.V, cfg.pad_idx, a.loss_row,
                reinterpret_cast<bf16*>(a.dlogits), s);
    } else {
      linear(dec_out(), dd, L.Wc, dd, a.logits, L.V, DType::F32, Md, L.V, dd, P(L.bc), 0, s);
      cross_entropy_rows(a.logits, a.tgt, Md, L.V, cfg.pad_idx, a.loss_row, a.dlogits, act, s);
    }
    float* lo = loss_out ? loss_out : a.loss;
    last_loss = lo;
    if (comm) {
      // data parallel: the mean CE over the GLOBAL batch (model.py:76) is the sum of the ranks'
      // partial sums / global count -- one 4-byte all-reduce, then the (Focal) loss and the
      // gradient scale from it on every rank (FocalLoss transforms the global mean, loss.py:20-28)
      loss_finalize(a.loss_row, Md, a.count, 0, a.loss_ce, nullptr, s, nullptr, /*partial=*/1);
      nccl_op(s, "allreduce(ce)", a.loss_ce, 4);
      NCCL_CHECK(ncclAllReduce(a.loss_ce, a.loss_ce, 1, ncclFloat, ncclSum, comm, s));
      loss_finalize(nullptr, 0, a.count, cfg.focal_loss, lo, a.grad_scale, s, a.loss_ce);
    } else if (!defer) {
      loss_finalize(a.loss_row, Md, a.count, cfg.focal_loss, lo, a.grad_scale, s);
    }
    stamp_fwd_end = stamp_next;
  }

  // ------------------------------------------------------------------------------------
  // weight-gradient GEMMs run on the side stream es2, forked from the main stream right after
  // their inputs are produced; backward() joins es2 back at the end (both in eager mode and
  // inside the captured graph, where this becomes a parallel branch)
  // `to` waits for everything issued so far on `from` (no-op when they are one stream)
  static void dep(hipStream_t from, hipStream_t to, hipEvent_t e) {
    if (from == to) return;
    hz::record(e, from);
    hz::wait(to, e);
  }
  static void memset_async(void* p, size_t bytes, hipStream_t s) {
    if (hz::active()) hz::op(s, "memset", {hz::wr(p, (int64_t)bytes)});
    CAPGEN_HIP(hipMemsetAsync(p, 0, bytes, s));
  }
  // an RCCL collective on s, in place over [p, p + bytes): hazard log + the collective log
  // (capgen_debug_collectives: every rank must issue the same sequence, or the job hangs)
  bool coll_log_on = false;
  std::vector<std::string> coll_log;
  void nccl_op(hipStream_t s, const char* name, const void* p, int64_t bytes) {
    if (hz::g_log) hz::op(s, name, {hz::wr(p, bytes)});
    if (coll_log_on) {
      const char* role = s == ec ? "bucket" : s == es2 ? "side" : "critical";
      coll_log.push_back(std::string(name) + " " + std::to_string(bytes) + " B on " + role);
    }
  }
  void fork(hipStream_t s) { dep(s, es2, ev_fork); }
  void join(hipStream_t s) {
    flush(s);
    if (!dbg_drop_join) dep(es2, s, ev_join);
  }
  // hazard-checker self-test (CAPGEN_DEBUG_DROP_JOIN=1): the side stream is never joined back --
  // a deliberately missing edge the checker must report (results are then racy: test use only)
  bool dbg_drop_join = knob(Knob::DebugDropJoin) == 1;  // (debug build only)
  // Weight-gradient GEMMs are queued and issued on es2 in one batch per block (flush): an event
  // record/wait pair costs the recording stream ~7 us of bubble on ROCm 7 (tools/kprobe.hip:
  // 13 us per eager fork/join pair), so the critical stream records one event per block instead
  // of one per weight.  Every buffer a queued dW reads is per block (or never rewritten in the
  // backward pass), so issuing it later is hazard-free.
  struct DwJob {
    const void *dY, *X;
    int64_t ldy, ldx, goff, ldg;
    int M, N, K;
    const float* alpha_ptr;
  };
  std::vector<DwJob> dw_pending;
  bool group_dw = knob(Knob::GroupDw) != 0;  // 0: one launch per weight (tests)
  void dw_side(const void* dY, int64_t ldy, const void* X, int64_t ldx, int64_t goff, int64_t ldg, int M, int N,
               int K, const float* alpha_ptr, hipStream_t s) {
    if (es2 == s) {
      linear_dw(dY, ldy, X, ldx, goff, ldg, M, N, K, alpha_ptr, s);
      return;
    }
    dw_pending.push_back(DwJob{dY, X, ldy, ldx, goff, ldg, M, N, K, alpha_ptr});
  }
  GemmArgs dw_args(const DwJob& j) const {
    GemmArgs ga;
    ga.M = j.N, ga.N = j.K, ga.K = j.M, ga.A = j.dY, ga.lda = j.ldy, ga.B = j.X, ga.ldb = j.ldx;
    ga.C = G(j.goff), ga.ldc = j.ldg, ga.alpha_ptr = j.alpha_ptr;
    return ga;
  }
  // run weight-gradient jobs on stream st now: in bf16 mode as grouped launches (every dW tile
  // of a block in one grid: better chip fill than 4-6 small launches, tools/dw_variant_probe.sh)
  void dw_launch(const DwJob* jobs, size_t n, hipStream_t st) {
    if (act == DType::BF16 && group_dw) {
      std::vector<GemmArgs> probs;
      for (size_t i = 0; i < n; ++i) probs.push_back(dw_args(jobs[i]));
      for (size_t i = 0; i < n; i += kMaxGroup) {
        if (stamp_on) probs[i].stamp = stamp(st, "gemm dW group of " + std::to_string(std::min<size_t>(kMaxGroup, n - i)));
        gemm_grouped(probs.data() + i, (int)std::min<size_t>(kMaxGroup, n - i), DType::F32, true, true, st);
      }
    } else {
      for (size_t i = 0; i < n; ++i) {
        const DwJob& j = jobs[i];
        linear_dw(j.dY, j.ldy, j.X, j.ldx, j.goff, j.ldg, j.M, j.N, j.K, j.alpha_ptr, st);
      }
    }
  }
  // FFN bias gradients (column sums of the ReLU'-masked hidden gradient) queued like the weight
  // gradients: off the critical stream instead of as atomics in the dX GEMM's epilogue
  // (CAPGEN_COLSUM_SIDE=0 restores the epilogue form)
  struct ColJob {
    const void* X;
    int M, N;
    float* db;
  };
  std::vector<ColJob> col_pending;
  bool colsum_side = knob(Knob::ColsumSide) != 0;
  // es2 waits for everything issued on s so far, then runs the queued weight-gradient GEMMs
  void flush(hipStream_t s) {
    fork(s);
    dw_launch(dw_pending.data(), dw_pending.size(), es2);
    dw_pending.clear();
    for (const ColJob& j : col_pending) column_sum(j.X, j.M, j.N, j.N, 1.f, nullptr, j.db, act, es2, NSTRIPE, n_small);
    col_pending.clear();
  }
  // Decoder block 0's self-attention half (and the decoder-embedding branch) on es2, concurrent
  // with the encoder chain: once block 0's cross-attention backward has produced its K/V
  // gradient, the encoder-output gradient (all blocks' gKV . Wkv_all) is complete, and nothing
  // the encoder backward reads depends on the rest of block 0 (CAPGEN_OVERLAP_DEC0=0: serial)
  bool overlap_front = knob(Knob::OverlapFront) != 0;  // 0: the decoder front runs after the encoder
  bool overlap_dec0 = knob(Knob::OverlapDec0) != 0;
  // GemmArgs of dX[M,K] (+)= dY[M,N] . W[N,K] (linear_dx) without launching it
  GemmArgs dx_args(const void* dY, int64_t ldy, int64_t woff, int64_t ldw, void* dX, int64_t ldx, int M, int N,
                   int K, int beta) const {
    GemmArgs ga;
    ga.M = M, ga.N = K, ga.K = N, ga.A = dY, ga.lda = ldy, ga.B = W(woff), ga.ldb = ldw, ga.C = dX, ga.ldc = ldx;
    ga.beta = beta;
    return ga;
  }

  // lb = the block's LayerNorm backward (dy = grad wrt block output, d_res -> r_out, d_a -> gA);
  // X = block input, H = hidden activations.
  void ffn_bwd(int M, int d, int f, const LnBwd& lb, const void* X, const void* H, int64_t W1, int64_t b1, int64_t W2,
               void* gH, hipStream_t s) {
    lnb(lb, s);
    void* gA = lb.d_a;
    dw_side(gA, d, H, f, W2, f, M, d, f, nullptr, s);
    const bool side = colsum_side && es2 != s;
    linear_dx(gA, d, W2, f, gH, f, M, d, f, 0, H, nullptr, s, side ? nullptr : GS(b1));  // x relu'(H)
    if (side) col_pending.push_back(ColJob{gH, M, f, GS(b1)});                           // db1 = colsum
    dw_side(gH, f, X, d, W1, d, M, f, d, nullptr, s);
    linear_dx(gH, f, W1, d, lb.d_res, d, M, f, d, 1, nullptr, nullptr, s);
  }
  // MHA output projection + LayerNorm backward: lb as above (d_res = grad wrt the residual /
  // query input); writes grad wrt the attention output into gATT.
  void mha_out_bwd(int M, int d, const LnBwd& lb, const void* att, int64_t Wo, void* gATT, hipStream_t s) {
    lnb(lb, s);
    dw_side(lb.d_a, d, att, d, Wo, d, M, d, d, nullptr, s);
    linear_dx(lb.d_a, d, Wo, d, gATT, d, M, d, d, 0, nullptr, nullptr, s);
  }
  // ... followed by the attention backward of g: in bf16 with the tiled Wo^T, the projection's input
  // gradient (dO = dA . Wo, dA = lb.d_a) runs INSIDE the attention backward launch (qkv_attn_bwd):
  // one launch and one dependent boundary fewer per attention block (CAPGEN_FUSED_ATTN_BWD=0: the
  // dX GEMM into gATT and the attention backward launch)
  bool fused_attn_bwd_on = knob(Knob::FusedAttnBwd) != 0;
  void mha_bwd(int M, int d, const LnBwd& lb, const void* att, int64_t Wo, void* gATT, const AttnGeom& g,
               const float* probs, void* dq, void* dk, void* dv, hipStream_t s) {
    if (fused_attn_bwd_on && act == DType::BF16 && WTo(Wo) && attention_mfma_ok(g)) {
      QkvBwd qb;
      qb.g = g, qb.g.prio = prio(s);
      qb.dA = reinterpret_cast<const bf16*>(lb.d_a), qb.ldda = d, qb.Wt = WTo(Wo);
      qb.dq = reinterpret_cast<bf16*>(dq), qb.dk = reinterpret_cast<bf16*>(dk), qb.dv = reinterpret_cast<bf16*>(dv);
      if (qkv_bwd_ok(qb)) {
        lnb(lb, s);
        dw_side(lb.d_a, d, att, d, Wo, d, M, d, d, nullptr, s);
        if (stamp_on) qb.g.stamp = stamp(s, "attn_bwd_wo " + std::to_string(g.Lq) + "x" + std::to_string(g.Lk));
        qkv_attn_bwd(qb, s);
        return;
      }
    }
    mha_out_bwd(M, d, lb, att, Wo, gATT, s);
    attb(g, probs, gATT, dq, dk, dv, act, s);
  }

  // Adam over arena ranges; ranges are 64-element aligned so the bf16 shadow slices line up
  void adam_range(int64_t off, int64_t n, hipStream_t s, int grid_cap = 0) {
    ++wver;  // (the embedding table has no shadow: its bf16 decode copy follows the version too)
    const int64_t ns = shadow ? std::max<int64_t>(0, std::min(n, L.n_dense - off)) : 0;
    // the fronts' tiled weights in this range: written by the Adam kernel itself (else re-tiled after)
    AdamTiles at;
    bool fused_tiles = true;
    for (auto& kv : tiled)
      if (ns > 0 && kv.second.second > 0 && kv.first < off + ns && kv.first + (int64_t)kv.second.second * 512 > off) {
        // a tiled matrix only partly inside this range (a bucket boundary through it): re-tile after
        if (at.n == AdamTiles::kMax || kv.first < off || kv.first + (int64_t)kv.second.second * 512 > off + ns ||
            (kv.first - off) % 4 != 0) {
          fused_tiles = false;
          break;
        }
        at.off[at.n] = kv.first - off, at.len[at.n] = (int64_t)kv.second.second * 512;
        at.dst[at.n++] = wtile + kv.second.first;
      }
    adam_update(params + off, grads + off, am + off, av + off, (size_t)n, cfg.beta1, cfg.beta2, cfg.eps, adam_scal,
                ns > 0 ? shadow + off : nullptr, (size_t)ns, s, grid_cap, fused_tiles ? at : AdamTiles{});
    if (ns > 0) retile(off, ns, s, /*trans_only=*/fused_tiles);  // (the transposed ones: always a launch)
  }
  // Adam grid of the step's last buckets (embedding, encoder LN/biases), which sit between the
  // backward's end and the next forward: the common cap (0).  The whole chip for them measured
  // slower (4-round A/B: 3.012 vs 2.982 ms/step with 2048 vs 256 workgroups)
  static constexpr int tail_grid = 0;

  // Step mode (train_step): the parameter update is bucketed.  A bucket is an arena range
  // whose gradients are final and whose weights nothing later in the backward pass reads
  // (one transformer block, the classifier, ...).  When backward reaches that point, the
  // bucket stream ec waits for both compute streams, all-reduces the bucket's gradients
  // over RCCL (DP) and runs Adam on it, overlapped with the rest of the backward pass.
  // Buckets are issued in reverse layer order: 12-20 MB each at C2, one per block.
  // sync: first flush (es2 waits for s, queued dW issued); sync=false when es2 already holds
  // every producer of the bucket's gradients (consecutive buckets after one flush)
  // from_s: every producer of the bucket's gradients ran on s (no flush, ec waits for s)
  bool bstep = false;
  // transformer blocks per gradient bucket (one flush = one event record on the critical stream)
  int bucket_blocks = std::max(1, knob(Knob::BucketBlocks));
  void bucket(int64_t off, int64_t n, hipStream_t s, bool sync = true, bool from_s = false) {
    if (sync && !from_s) flush(s);
    if (!bstep) return;
    if (from_s) dep(s, ec, ev_b1);
    else dep(es2, ec, ev_b2);
    bucket_update(off, n);
  }
  // the bucket's all-reduce (DP) + Adam on the bucket stream (its producers already waited for)
  void bucket_update(int64_t off, int64_t n, int grid_cap = 0) {
    ++wver;
    zbuckets.push_back({off, n});
    const int zw = zworld();
    if (zsharded() && n % (4 * zw) == 0) {  // sharded update (ZeRO-1); buckets are 64-element aligned
      const int64_t c = n / zw, o = off + (int64_t)zrank() * c;
      if (zw > 1) moments_sharded = true;  // this rank's moments are current in its chunks only
      if (comm && zw > 1) grads_sharded = true;  // the gradient arena holds reduce-scattered chunks
      // in place: rank r's chunk of the summed gradients lands at grads + o
      if (comm) {
        nccl_op(ec, "reduce_scatter", grads + off, n * 4);
        NCCL_CHECK(ncclReduceScatter(grads + off, grads + o, (size_t)c, ncclFloat, ncclSum, comm, ec));
      }
      const int64_t ns = shadow ? std::max<int64_t>(0, std::min(n, L.n_dense - off)) : 0;
      adam_update(params + o, grads + o, am + o, av + o, (size_t)c, cfg.beta1, cfg.beta2, cfg.eps, adam_scal, nullptr, 0,
                  ec, grid_cap);
      // in place: every rank's updated chunk -> params + off (sendbuff = recvbuff + rank * c)
      if (comm) {
        nccl_op(ec, "all_gather", params + off, n * 4);
        NCCL_CHECK(ncclAllGather(params + o, params + off, (size_t)c, ncclFloat, comm, ec));
      }
      if (ns > 0) to_bf16(params + off, shadow + off, (size_t)ns, ec);
      if (ns > 0) retile(off, ns, ec);
      return;
    }
    if (comm) {
        nccl_op(ec, "allreduce(bucket)", grads + off, n * 4);
        NCCL_CHECK(ncclAllReduce(grads + off, grads + off, (size_t)n, ncclFloat, ncclSum, comm, ec));
      }
    adam_range(off, n, ec, grid_cap);
  }
  // once: the step's buckets cover the arena exactly (each element updated by exactly one bucket)
  void check_buckets() {
    if (zbuckets_checked) return;
    auto v = zbuckets;
    std::sort(v.begin(), v.end());
    int64_t end = 0;
    for (auto& b : v) {
      require(b[0] == end && b[1] > 0, "internal: gradient buckets do not tile the parameter arena");
      end = b[0] + b[1];
    }
    require(end == L.total, "internal: gradient buckets do not cover the parameter arena");
    zbuckets_checked = true;
  }
  int64_t enc_end(int l) const { return l + 1 < L.Le ? L.enc[l + 1].Wqkv : L.Wel; }
  int64_t dec_end(int l) const { return l + 1 < L.Ld ? L.dec[l + 1].Wqkv : L.Wkv_all; }

  // backward of enc_layer_fwd: gO = grad wrt Xout on entry, grad wrt X on exit; gR scratch
  void enc_layer_bwd(const EncLayerOff& w, EncAct& A, Acts::GradBufs& gb, const void* X, int B, int N,
                     const uint8_t* valid, int layer, bool on, void* gO, void* gR, hipStream_t s) {
    const int Me = B * N, d = L.d, He = L.He, dke = d / He;
    void* go = gO;
    const float p = cfg.dropout, pa = cfg.attention_dropout;
    RowMask mask{};
    mask.valid = valid;
    const LnBwd lffn = lnb_desc(Me, d, gO, A.v2, A.m2, A.r2, w.ln2g, w.ln2b, w.b2, mask, mk_drop(p, site(0, layer, 2), on),
                                gR, gb.gAf);
    const LnBwd lmha = lnb_desc(Me, d, gR, A.v1, A.m1, A.r1, w.ln1g, w.ln1b, -1, RowMask{},
                                mk_drop(p, site(0, layer, 1), on), go, gb.gA1);
    ffn_bwd(Me, d, L.fe, lffn, A.Y, A.H, w.W1, w.b1, w.W2, gb.gH, s);  // gR = grad wrt Y
    AttnGeom g;
    g.B = B, g.H = He, g.Lq = N, g.Lk = N, g.dk = dke;
    g.q = A.qkv, g.q_ld = 3 * d, g.q_bs = (int64_t)N * 3 * d;
    g.k = at(A.qkv, d), g.k_ld = 3 * d, g.k_bs = (int64_t)N * 3 * d;
    g.v = at(A.qkv, 2 * d), g.v_ld = 3 * d, g.v_bs = (int64_t)N * 3 * d;
    g.o_ld = d, g.o_bs = (int64_t)N * d;
    if (valid) g.key_valid = valid, g.kv_bs = N, g.causal = 1;
    g.temperature = std::sqrt((float)dke);
    g.drop = mk_drop(pa, site(0, layer, 0), on);
    mha_bwd(Me, d, lmha, A.att, w.Wo, gb.gATT1, g, A.P, gb.gQKV, at(gb.gQKV, d), at(gb.gQKV, 2 * d), s);
    dw_side(gb.gQKV, 3 * d, X, d, w.Wqkv, d, Me, 3 * d, d, nullptr, s);
    linear_dx(gb.gQKV, 3 * d, w.Wqkv, d, go, d, Me, 3 * d, d, 1, nullptr, nullptr, s);  // gO = grad wrt X
  }

  // backward of image_objects_fwd: gX0 = grad wrt a.X[0] -> embedding weight gradient
  void image_objects_bwd(const void* gX0, int B, int N, bool on, hipStream_t s) {
    const int Me = B * N, d = L.d;
    // second norm: grad wrt Z[2r+1] + Ep[r] (no residual, no dropout)
    lnb(lnb_desc(Me, d, gX0, a.siV, a.siM, a.siR, L.enc_lng, L.enc_lnb, -1, RowMask{}, Drop{}, nullptr,
                           a.siGEp), s);
    pair_scatter(a.siGEp, Me, d, a.siG0, act, s);  // only the region token's output is kept
    enc_layer_bwd(L.img, a.si, a.gsi, a.siX2, Me, 2, a.siValid, kImgLayer, on, a.siG0, a.siG1, s);
    pair_reduce(a.siG0, B, N, d, a.siGY, act, s);  // image-row tokens fold back onto region 0
    lnb(lnb_desc(Me, d, a.siGY, a.ev0, a.em0, a.er0, L.enc_lng, L.enc_lnb, -1, RowMask{}, Drop{}, nullptr,
                           a.gAe), s);
    // feature columns see the first embedding only; position columns both (+ Ep after the block)
    linear_dw(a.gAe, d, a.Aenc, L.Kp, L.enc_emb_W, L.Kp, Me, d, L.F, nullptr, s);
    add_inplace(a.siGEp, a.gAe, (int64_t)Me * d, act, s);
    linear_dw(a.siGEp, d, at(a.Aenc, L.F), L.Kp, L.enc_emb_W + L.F, L.Kp, Me, d, L.Kp - L.F, nullptr, s);
  }

  // backward of move_first_fwd at the training shape (dy = a.gOut): a.gRes = grad wrt D[Ld]
  // (residual + U), a.mfGU = grad wrt U
  void move_first_bwd(int Md, bool on, hipStream_t s) {
    const int dd = L.dd, fd = L.fd;
    const LnBwd lb = lnb_desc(Md, dd, a.gOut, a.mfV, a.mfM, a.mfR, L.mf_lng, L.mf_lnb, L.mf_b2, RowMask{},
                              mk_drop(cfg.dropout, site(1, kMfLayer, 0), on), a.gRes, a.mfGA);
    lnb(lb, s);
    dw_side(a.mfGA, dd, a.mfH, fd, L.mf_W2, fd, Md, dd, fd, nullptr, s);
    linear_dx(a.mfGA, dd, L.mf_W2, fd, a.mfGH, fd, Md, dd, fd, 0, a.mfH, nullptr, s, GS(L.mf_b1));
    dw_side(a.mfGH, fd, a.mfU, dd, L.mf_W1, dd, Md, fd, dd, nullptr, s);
    linear_dx(a.mfGH, fd, L.mf_W1, dd, a.mfGU, dd, Md, fd, dd, 0, nullptr, nullptr, s);
    add_inplace(a.gRes, a.mfGU, (int64_t)Md * dd, act, s);
  }

  // step_params: bucketed all-reduce + Adam (see bucket()); otherwise gradients only
  bool dec0_on_side = false;  // backward(): decoder block 0 was issued on es2 (overlap_dec0)
  void backward(hipStream_t s, bool step_params = false) {
    bstep = step_params;
    require(fB > 0, "backward: call forward first");
    grads_sharded = false;
    stamp_next = stamp_fwd_end;
    const int B = fB, N = fN, Lq = fT - 1, Me = B * N, Md = B * Lq, d = L.d, dd = L.dd;
    const int He = L.He, Hd = L.Hd, dke = d / He, dkd = dd / Hd;
    const bool on = fwd_drop;
    const float p = cfg.dropout, pa = cfg.attention_dropout;
    // the striped LN/bias partials start at 0 (the critical stream's first LayerNorm backward adds
    // into them); the accumulated word-embedding gradient (20 MB at C2) is zeroed on es2 after the
    // fork below -- its only writer is the embedding scatter on es2
    const bool emb_zero_side = es2 != s && !L.has_img && !L.has_mf;
    if (!emb_zero_side) memset_async(grads + L.n_dense, (L.enc_lng - L.n_dense) * sizeof(float), s);
    // the striped partials are cleared by the previous backward's folds (stripe_reduce(clear)); a
    // backward that did not reach both folds (diagnostic stops, errors) leaves them marked dirty
    if (stripes_dirty || !stripe_clear) memset_async(gstripe, (size_t)NSTRIPE * n_small * sizeof(float), s);
    stripes_dirty = true;
    int folds = 0;
    if (bstep) {
      // the step counter / bias corrections only feed the bucket stream's Adam: issue them there
      // (off the critical stream) unless the step is being captured (ec joins a capture only
      // through the buckets' events)
      hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
      CAPGEN_HIP(hipStreamIsCapturing(s, &cst));
      adam_prepare(step, cfg.lr, cfg.beta1, cfg.beta2, adam_scal, cst == hipStreamCaptureStatusNone ? ec : s);
      zbuckets.clear();
    }

    RowMask dmask{};
    dmask.ids = a.ids, dmask.pad_idx = cfg.pad_idx;
    // the LayerNorm backward of every block (model.py:86-90, 114-120 restated backward)
    auto dec_ffn_lb = [&](int l, const void* dy, void* dres) {
      const auto& A = a.dec[l];
      const auto& w = L.dec[l];
      return lnb_desc(Md, dd, dy, A.vf, A.mf, A.rf, w.lfg, w.lfb, w.b2, dmask, mk_drop(p, site(1, l, 7), on), dres,
                      a.gdec[l].gAf);
    };
    auto dec_cross_lb = [&](int l, const void* dy, void* dres) {
      const auto& A = a.dec[l];
      const auto& w = L.dec[l];
      return lnb_desc(Md, dd, dy, A.vc, A.mc, A.rc, w.lcg, w.lcb, -1, RowMask{}, mk_drop(p, site(1, l, 6), on), dres,
                      a.gdec[l].gA2);
    };
    auto dec_self_lb = [&](int l, const void* dy, void* dres) {
      const auto& A = a.dec[l];
      const auto& w = L.dec[l];
      return lnb_desc(Md, dd, dy, A.vs, A.ms, A.rs, w.lsg, w.lsb, -1, RowMask{}, mk_drop(p, site(1, l, 4), on), dres,
                      a.gdec[l].gA1);
    };
    auto dec_emb_lb = [&](const void* dy) {  // LN(E.Wel^T + PE) (model.py:432-436): no residual, no dropout
      return lnb_desc(Md, dd, dy, a.dv0, a.dm0, a.dr0, L.dec_lng, L.dec_lnb, -1, RowMask{}, Drop{}, nullptr, a.gAd);
    };
    auto enc_emb_lb = [&](const void* dy) {
      return lnb_desc(Me, d, dy, a.ev0, a.em0, a.er0, L.enc_lng, L.enc_lnb, -1, RowMask{}, Drop{}, nullptr, a.gAe);
    };

    // classifier: dlogits are unscaled (softmax - onehot); grad_scale folds 1/count (+focal).  The
    // critical stream goes straight from the forward into the dX GEMM: the side work (weight and bias
    // gradients, the embedding-gradient clear, a deferred loss finalisation) forks after it, with the
    // flush the classifier's bucket needs anyway (one event record on the critical stream, not two)
    dw_side(a.dlogits, L.V, dec_out(), dd, L.Wc, dd, Md, L.V, dd, a.grad_scale, s);
    linear_dx(a.dlogits, L.V, L.Wc, dd, a.gOut, dd, Md, L.V, dd, 0, nullptr, a.grad_scale, s);
    flush(s);  // es2: the classifier dW (the bucket below waits for it: it reads Wc's gradient)
    bucket(L.Wc, L.n_dense - L.Wc, s, /*sync=*/false);
    if (emb_zero_side) memset_async(grads + L.n_dense, (L.enc_lng - L.n_dense) * sizeof(float), es2);
    column_sum(a.dlogits, Md, L.V, L.V, 1.f, a.grad_scale, GS(L.bc), act, es2, NSTRIPE, n_small);
    if (pending_loss) {  // the mean CE (model.py:96); grad_scale was written by the caption prep
      loss_finalize(a.loss_row, Md, a.count, 0, pending_loss, nullptr, es2);
      pending_loss = nullptr;
    }

    const int64_t kvld = (int64_t)L.Ld * 2 * dd;
    void* gO = a.gOut;
    void* gR = a.gRes;
    if (L.has_mf) {  // gRes = grad wrt D[Ld]; a.mfGU = grad wrt U (its encoder part is added below)
      move_first_bwd(Md, on, s);
      std::swap(gO, gR);
    }
    for (int l = L.Ld - 1; l >= 0; --l) {
      const auto& w = L.dec[l];
      auto& A = a.dec[l];
      auto& gb = a.gdec[l];
      const LnBwd lffn = dec_ffn_lb(l, gO, gR), lcross = dec_cross_lb(l, gR, gO), lself = dec_self_lb(l, gO, gR);
      ffn_bwd(Md, dd, L.fd, lffn, A.D2, A.H, w.W1, w.b1, w.W2, gb.gH, s);  // gR = grad wrt D2
      AttnGeom c;
      c.B = B, c.H = Hd, c.Lq = Lq, c.Lk = N, c.dk = dkd;
      c.q = A.qc, c.q_ld = dd, c.q_bs = (int64_t)Lq * dd;
      c.k = at(a.KV, (int64_t)l * 2 * dd), c.k_ld = kvld, c.k_bs = (int64_t)N * kvld;
      c.v = at(a.KV, (int64_t)l * 2 * dd + dd), c.v_ld = kvld, c.v_bs = (int64_t)N * kvld;
      c.o_ld = dd, c.o_bs = (int64_t)Lq * dd;
      c.key_valid = a.valid, c.kv_bs = N;  // masks as in forward (the MFMA backward recomputes P)
      c.temperature = std::sqrt((float)dkd);
      c.drop = mk_drop(pa, site(1, l, 5), on);
      // (lcross.d_res = grad wrt D1, the residual part)
      mha_bwd(Md, dd, lcross, A.attc, w.Wo_c, gb.gATT2, c, A.Pc, gb.gQc, at(a.gKV, (int64_t)l * 2 * dd),
              at(a.gKV, (int64_t)l * 2 * dd + dd), s);
      // block 0: the rest of the block runs on es2 (ov), the encoder chain starts on s below
      const bool ov = l == 0 && overlap_dec0 && es2 != s;
      const hipStream_t hs = ov ? es2 : s;
      if (ov) flush(s);  // es2 waits for block 0's cross-attention backward; queued dW issued
      dw_side(gb.gQc, dd, A.D1, dd, w.Wq_c, dd, Md, dd, dd, nullptr, hs);
      linear_dx(gb.gQc, dd, w.Wq_c, dd, gO, dd, Md, dd, dd, 1, nullptr, nullptr, hs);  // gO = grad wrt D1
      AttnGeom g;
      g.B = B, g.H = Hd, g.Lq = Lq, g.Lk = Lq, g.dk = dkd;
      g.q = A.qkv, g.q_ld = 3 * dd, g.q_bs = (int64_t)Lq * 3 * dd;
      g.k = at(A.qkv, dd), g.k_ld = 3 * dd, g.k_bs = (int64_t)Lq * 3 * dd;
      g.v = at(A.qkv, 2 * dd), g.v_ld = 3 * dd, g.v_bs = (int64_t)Lq * 3 * dd;
      g.o_ld = dd, g.o_bs = (int64_t)Lq * dd;
      g.key_ids = a.ids, g.kid_bs = Lq, g.pad_idx = cfg.pad_idx, g.causal = 1;  // as in forward
      g.temperature = std::sqrt((float)dkd);
      g.drop = mk_drop(pa, site(1, l, 3), on);
      // (lself.d_res = grad wrt D_l, the residual part)
      mha_bwd(Md, dd, lself, A.atts, w.Wo_s, gb.gATT1, g, A.Ps, gb.gQKV, at(gb.gQKV, dd), at(gb.gQKV, 2 * dd), hs);
      dw_side(gb.gQKV, 3 * dd, a.D[l], dd, w.Wqkv, dd, Md, 3 * dd, dd, nullptr, hs);
      linear_dx(gb.gQKV, 3 * dd, w.Wqkv, dd, gR, dd, Md, 3 * dd, dd, 1, nullptr, nullptr, hs);
      if (l % bucket_blocks == 0)  // blocks l .. l + bucket_blocks - 1 (contiguous in the arena)
        (ov || l == 0 ? bucket(w.Wqkv, dec_end(std::min(l + bucket_blocks - 1, L.Ld - 1)) - w.Wqkv, hs)
                      : bucket(w.Wqkv, dec_end(std::min(l + bucket_blocks - 1, L.Ld - 1)) - w.Wqkv, hs));
      if (ov) dec0_on_side = true;
      std::swap(gO, gR);  // gO = grad wrt D_l
    }
    // cross K/V of all decoder blocks -> encoder output (the encoder chain starts here; the
    // Wkv_all weight gradient is queued after the dX GEMM below, which reads Wkv_all)
    // the buffer gO is not using -- or, with block 0 finishing on es2 (both in use there), gEnc
    void* eO = dec0_on_side ? a.gEnc : gO == a.gOut ? a.gRes : a.gOut;
    dec0_on_side = false;
    // decoder embedding: LN(E.Wel^T + PE) (model.py:432-436) -- off the critical path
    {
      const LnBwd lb = dec_emb_lb(gO);
      flush(s);
      lnb(lb, es2);
      linear_dx(a.gAd, dd, L.Wel, L.dwe, a.gE, L.dwe, Md, dd, L.dwe, 0, nullptr, nullptr, es2);
      const DwJob wel{a.gAd, a.E, dd, L.dwe, L.Wel, L.dwe, Md, dd, L.dwe, nullptr};
      dw_launch(&wel, 1, es2);
      embedding_scatter_add(a.gE, a.ids, Md, L.dwe, cfg.pad_idx, G(L.emb), act, es2, L.V);
      // every decoder-side gradient is final here (in es2 order, after the fork above)
      stripe_reduce(GS(L.dec_lng), NSTRIPE, n_small, L.total - L.dec_lng, G(L.dec_lng), 0, es2, stripe_clear);
      ++folds;
    }
    // the encoder chain must not overwrite gO (read by the decoder-embedding branch on es2):
    // it runs on the other residual buffer and on tmp (free during backward)
    gO = eO;
    gR = a.tmp;
    linear_dx(a.gKV, kvld, L.Wkv_all, d, gO, d, Me, L.Ld * 2 * dd, d, 0, nullptr, nullptr, s);
    if (L.has_mf) first_region_grad(a.mfGU, B, Lq, N, d, gO, act, s);  // enc[:, 0] of U = D + enc[:, 0]
    dw_side(a.gKV, kvld, a.X[L.Le], d, L.Wkv_all, d, Me, L.Ld * 2 * dd, d, nullptr, s);
    // the decoder-embedding branch (es2) has been issued: every decoder-side gradient is final
    // the flush of the first bucket follows the dX GEMM above (it reads Wkv_all); es2 then holds
    // every producer of the other three buckets
    bucket(L.Wkv_all, L.Wc - L.Wkv_all, s);               // cross K/V of all decoder blocks
    bucket(L.Wel, L.dec[0].Wqkv - L.Wel, s, false);       // word-embedding projection
    bucket(L.emb, L.enc_lng - L.emb, s, false);           // word embedding table
    bucket(L.dec_lng, L.total - L.dec_lng, s, false);     // decoder LN / biases, classifier bias
    for (int l = L.Le - 1; l >= 0; --l) {
      const auto& w = L.enc[l];
      enc_layer_bwd(w, a.enc[l], a.genc[l], a.X[l], B, N, cfg.encode_mask ? a.valid : nullptr, l, on, gO, gR, s);
      if (l % bucket_blocks == 0)
        (l == 0 ? bucket(w.Wqkv, enc_end(std::min(l + bucket_blocks - 1, L.Le - 1)) - w.Wqkv, s)
                : bucket(w.Wqkv, enc_end(std::min(l + bucket_blocks - 1, L.Le - 1)) - w.Wqkv, s));
    }
    // the tail of the step's dependency chain: the encoder-embedding LayerNorm backward and
    // weight gradient, then its Adam, which the next forward's first GEMM needs -- on the
    // critical stream, so it does not queue behind the weight-gradient groups still on es2
    // (a single GEMM: the plain launch with its autotuned split-K, K = B*N = 2304 deep)
    if (L.has_img) {
      image_objects_bwd(gO, B, N, on, s);
      flush(s);  // the image block's weight gradients share the embedding bucket
    } else {
      lnb(enc_emb_lb(gO), s);
      linear_dw(a.gAe, d, a.Aenc, L.Kp, L.enc_emb_W, L.Kp, Me, d, L.Kp, nullptr, s);
    }
    // every encoder LayerNorm/bias partial was accumulated on s; in step mode the fold and the
    // last two buckets (feature/position embedding, encoder LN / biases) run on the bucket
    // stream behind ONE event (each event record costs the critical stream ~5 us)
    const hipStream_t tail = bstep ? ec : s;
    if (!bstep) join(s);  // queued bias column sums (es2) precede the fold below
    if (bstep) dep(s, ec, ev_b1);
    if (bstep && L.has_img) dep(es2, ec, ev_b2);
    stripe_reduce(GS(L.enc_lng), NSTRIPE, n_small, L.dec_lng - L.enc_lng, G(L.enc_lng), 0, tail, stripe_clear);
    if (++folds == 2) stripes_dirty = false;
    if (bstep) {
      bucket_update(0, L.enc[0].Wqkv, tail_grid);                   // feature/position embedding
      bucket_update(L.enc_lng, L.dec_lng - L.enc_lng, tail_grid);   // encoder LN / biases
    }
    join(s);
    if (bstep) {
      dep(ec, s, ev_cj);
      bstep = false;
      check_buckets();
    }
  }

  void allreduce_grads(hipStream_t s) {
    if (!comm) return;
    nccl_op(s, "allreduce(grads)", grads, L.total * 4);
    NCCL_CHECK(ncclAllReduce(grads, grads, (size_t)L.total, ncclFloat, ncclSum, comm, s));
  }

  void adam(hipStream_t s) {
    ++wver;
    adam_prepare(step, cfg.lr, cfg.beta1, cfg.beta2, adam_scal, s);
    adam_update(params, grads, am, av, (size_t)L.total, cfg.beta1, cfg.beta2, cfg.eps, adam_scal, shadow,
                shadow ? (size_t)L.n_dense : 0, s);
    if (shadow) retile(0, L.n_dense, s);
  }

  void refresh_shadow(hipStream_t s) {
    if (shadow) to_bf16(params, shadow, (size_t)L.n_dense, s);
    if (shadow) retile(0, L.n_dense, s);
  }

  // ------------------------------------------------------------------------------------
  // stream hand-off: caller stream -> engine stream -> caller stream
  void enter(hipStream_t cs) {
    hz::record(ev_in, cs);
    hz::wait(es, ev_in);
    hz::set_critical(es);
  }
  void leave(hipStream_t cs) {
    hz::record(ev_out, es);
    hz::wait(cs, ev_out);
  }

  // Once, after the first train step at world > 1: every rank must hold the same GLOBAL non-pad count
  // (the count all-reduce inside the forward -- captured in its graph -- gives the reference's mean over
  // the global batch, model.py:76) and so the same loss.  Max and min over the ranks of both, one
  // grouped 4-value exchange; a mismatch fails the step (non-zero status, capgen_last_error).
  // `force` runs it regardless of world size and of an earlier check (capgen_dp_check: the world-1
  // rehearsal of the exchange; the step's own call passes false).  `loss` null = the loss buffer the
  // last forward wrote (its loss_out, or the internal one).
  bool dp_checked = false;
  float* dp_chk = nullptr;  // [4] device scratch: count max, count min, loss max, loss min
  const float* last_loss = nullptr;
  void dp_check(hipStream_t cs, const float* loss, bool force = false) {
    if (!comm || (!force && (dp_checked || world <= 1))) return;
    dp_checked = true;
    if (!dp_chk) CAPGEN_HIP(hipMalloc(&dp_chk, 4 * sizeof(float)));
    const float* lo = loss ? loss : last_loss;
    require(a.count && lo, "dp_check: no train step yet");
    for (int i = 0; i < 2; ++i) {
      CAPGEN_HIP(hipMemcpyAsync(dp_chk + i, a.count, sizeof(float), hipMemcpyDeviceToDevice, cs));
      CAPGEN_HIP(hipMemcpyAsync(dp_chk + 2 + i, lo, sizeof(float), hipMemcpyDeviceToDevice, cs));
    }
    NCCL_CHECK(ncclGroupStart());
    NCCL_CHECK(ncclAllReduce(dp_chk, dp_chk, 1, ncclFloat, ncclMax, comm, cs));
    NCCL_CHECK(ncclAllReduce(dp_chk + 1, dp_chk + 1, 1, ncclFloat, ncclMin, comm, cs));
    NCCL_CHECK(ncclAllReduce(dp_chk + 2, dp_chk + 2, 1, ncclFloat, ncclMax, comm, cs));
    NCCL_CHECK(ncclAllReduce(dp_chk + 3, dp_chk + 3, 1, ncclFloat, ncclMin, comm, cs));
    NCCL_CHECK(ncclGroupEnd());
    float hv[4];
    CAPGEN_HIP(hipMemcpyAsync(hv, dp_chk, sizeof hv, hipMemcpyDeviceToHost, cs));
    CAPGEN_HIP(hipStreamSynchronize(cs));
    require(hv[0] == hv[1] && hv[0] > 0.f,
            "dp: the global target count differs across ranks after the first step (max " + std::to_string(hv[0]) +
                ", min " + std::to_string(hv[1]) + ")");
    require(hv[2] == hv[3], "dp: the global loss differs across ranks after the first step (max " +
                                std::to_string(hv[2]) + ", min " + std::to_string(hv[3]) + ")");
  }

  // after a train step's forward (eager, captured or replayed): its deferred loss goes to `loss`
  void set_pending_loss(float* loss) {
    pending_loss = loss_deferrable() ? (loss ? loss : a.loss) : nullptr;
    if (pending_loss) last_loss = pending_loss;
  }
  void train_step(const void* f, DType ft, const float* pos, const int32_t* caps, int B, int N, int T, float* loss,
                  hipStream_t cs) {
    ensure_acts(B, N, T);
    Key k{f, pos, caps, loss, (int)ft, B, N, T, training, in_idx, in_n_img};
    // (the hazard checker's log runs the eager forward: the graph replays the same launches)
    const bool fwd_graph = fwd_graph_on && !hz::g_log && (world <= 1 || fwd_graph_mode == 2);
    if (direct_on && !graph_on && fwd_graph && !count_override && have_fwd_graph() && fkey == k && cs != es) {
      crit = cs;
      hz::set_critical(cs);
      launch_fwd(cs);
      fB = B, fN = N, fT = T, fwd_drop = training;  // host state forward() would have set
      set_pending_loss(loss);
      backward(cs, /*step_params=*/true);
      crit = nullptr;
      hz::record(ev_out, cs);
      hz::wait(es, ev_out);
      return;
    }
    enter(cs);
    auto body = [&]() {
      const bool host_timing = knob(Knob::HostTiming) != 0;  // (debug build)
      static double tf = 0, tb = 0;
      static int nsteps = 0;
      auto t0 = std::chrono::steady_clock::now();
      forward(f, ft, pos, caps, B, N, T, loss, training, es, /*defer_loss=*/true);
      set_pending_loss(loss);
      auto t1 = std::chrono::steady_clock::now();
      backward(es, /*step_params=*/true);  // + bucketed RCCL all-reduce (DP) and Adam
      if (host_timing) {
        auto t2 = std::chrono::steady_clock::now();
        tf += std::chrono::duration<double, std::micro>(t1 - t0).count();
        tb += std::chrono::duration<double, std::micro>(t2 - t1).count();
        if (++nsteps % 20 == 0) {
          std::fprintf(stderr, "[capgen host] enqueue per step: forward %.1f us, backward %.1f us\n", tf / 20, tb / 20);
          tf = tb = 0;
        }
      }
    };
    // under DP the forward graph holds the count and partial-CE all-reduces (RCCL ops capture);
    // a host-set global count (capgen_dp_set_global_count) runs the forward eagerly instead --
    // its pinned-memory copy must stay ordered against the host write
    if (!graph_on && fwd_graph && !count_override) {
      // forward replayed as one linear hipGraph (cheap to launch: ~0.1 us/node of host time vs
      // ~2.7 us per eager launch, tools/kprobe.hip); backward issued eagerly on three streams
      // (a multi-branch graph costs the same host time per node as eager issue on ROCm 7)
      if (!(have_fwd_graph() && fkey == k)) {
        drop_graph();
        if (!tuned(B, N, T)) {  // autotune every GEMM shape outside the capture
          forward(f, ft, pos, caps, B, N, T, loss, /*drop_on=*/false, es);
          backward(es);
          hz::host_sync(es);
          tuned_shapes.push_back({B, N, T});
        }
        hipGraph_t graph = nullptr;
        // split capture needs the decoder front on its own stream
        cap_split = fwd_split() && overlap_front && es2 != es;
        CAPGEN_HIP(hipStreamBeginCapture(es, hipStreamCaptureModeThreadLocal));
        try {
          forward(f, ft, pos, caps, B, N, T, loss, training, es, /*defer_loss=*/true);
        } catch (...) {
          (void)hipStreamEndCapture(es, &graph);
          if (graph) (void)hipGraphDestroy(graph);
          cap_split = false;
          for (auto& x : fg)
            if (x) (void)hipGraphDestroy(x), x = nullptr;
          throw;
        }
        CAPGEN_HIP(hipStreamEndCapture(es, &graph));
        if (cap_split) {
          fg[3] = graph;
          for (int i = 0; i < 4; ++i) {
            CAPGEN_HIP(hipGraphInstantiate(&fx[i], fg[i], nullptr, nullptr, 0));
            CAPGEN_HIP(hipGraphDestroy(fg[i]));
            fg[i] = nullptr;
          }
          cap_split = false;
        } else {
          CAPGEN_HIP(hipGraphInstantiate(&fexec, graph, nullptr, nullptr, 0));
          CAPGEN_HIP(hipGraphDestroy(graph));
        }
        fkey = k;
      }
      const bool host_timing = knob(Knob::HostTiming) != 0;  // (debug build)
      static double tb = 0, tl = 0;
      static int nsteps = 0;
      auto t0 = std::chrono::steady_clock::now();
      launch_fwd(es);
      auto t1 = std::chrono::steady_clock::now();
      fB = B, fN = N, fT = T, fwd_drop = training;  // host state forward() would have set
      set_pending_loss(loss);
      backward(es, /*step_params=*/true);
      if (host_timing) {
        auto t2 = std::chrono::steady_clock::now();
        tl += std::chrono::duration<double, std::micro>(t1 - t0).count();
        tb += std::chrono::duration<double, std::micro>(t2 - t1).count();
        if (++nsteps % 20 == 0) {
          std::fprintf(stderr, "[capgen host] per step: forward graph launch %.1f us, backward enqueue %.1f us\n",
                       tl / 20, tb / 20);
          tl = tb = 0;
        }
      }
    } else if (!graph_on) {
      body();
    } else {
      if (!(gexec && gkey == k)) {
        drop_graph();
        // one eager forward+backward (no all-reduce, no Adam) so every GEMM shape of the
        // step is autotuned outside the capture; its gradients are overwritten below
        if (!tuned(B, N, T)) {
          forward(f, ft, pos, caps, B, N, T, loss, /*drop_on=*/false, es);  // no RNG advance
          backward(es);
          hz::host_sync(es);
          tuned_shapes.push_back({B, N, T});
        }
        hipGraph_t graph = nullptr;
        CAPGEN_HIP(hipStreamBeginCapture(es, hipStreamCaptureModeThreadLocal));
        try {
          body();
        } catch (...) {
          (void)hipStreamEndCapture(es, &graph);
          if (graph) (void)hipGraphDestroy(graph);
          throw;
        }
        CAPGEN_HIP(hipStreamEndCapture(es, &graph));
        CAPGEN_HIP(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));
        CAPGEN_HIP(hipGraphDestroy(graph));
        gkey = k;
      }
      // the replay runs the captured Adam and re-cast of the shadow with no host code: the weight
      // version must move with it, or the decode tiles (build_dtiles) would keep the old weights
      ++wver;
      CAPGEN_HIP(hipGraphLaunch(gexec, es));
    }
    leave(cs);
  }

  // ------------------------------------------------------------------------------------
  // SCST (SelfCriticNetwork.train_step, models.py:179-195): rl_sample = teacher-forced forward,
  // PolicyNetwork.sample and the per-image entropy; the host scores the samples; rl_finish =
  // ReinforcementLearningLoss + backward + Adam.
  void rl_sample(const void* f, DType ft, const float* pos, const int32_t* caps, int B, int N, int T,
                 int64_t* sample_out, float* entropy_out, float* lm_out, hipStream_t cs) {
    ensure_acts(B, N, T);
    enter(cs);
    const int Lq = T - 1, Md = B * Lq;
    need_logits = true;  // rl_rows samples from the logits
    forward(f, ft, pos, caps, B, N, T, nullptr, training, es);
    need_logits = false;
    rl_rows(a.logits, Md, L.V, a.rl_sample, a.rl_lse, a.rl_logp, a.rl_ent, es);
    rl_image(a.rl_sample, a.rl_ent, B, Lq, a.rl_ent_img, a.rl_scal, es);
    if (sample_out) rl_export(a.rl_sample, Md, sample_out, es);
    if (entropy_out) CAPGEN_HIP(hipMemcpyAsync(entropy_out, a.rl_ent_img, B * sizeof(float), hipMemcpyDeviceToDevice, es));
    if (lm_out) CAPGEN_HIP(hipMemcpyAsync(lm_out, a.loss, sizeof(float), hipMemcpyDeviceToDevice, es));
    rl_B = B;
    leave(cs);
  }
  void rl_finish(const float* score, float w, float* out3, bool train, hipStream_t cs) {
    require(rl_B > 0 && rl_B == fB, "rl_finish: call rl_sample first");
    require(w >= 0.f && w <= 1.f, "rl_finish: structure_loss_weight must be in [0, 1]");
    enter(cs);
    const int B = fB, Lq = fT - 1;
    CAPGEN_HIP(hipMemcpyAsync(a.rl_score, score, B * sizeof(float), hipMemcpyDeviceToDevice, es));
    rl_numer(a.rl_sample, a.rl_logp, a.rl_score, B, Lq, a.rl_scal, es);
    if (comm) NCCL_CHECK(ncclAllReduce(a.rl_scal, a.rl_scal, 2, ncclFloat, ncclSum, comm, es));
    rl_loss(a.rl_scal, a.loss, w, out3 ? out3 : a.rl_scal + 2, a.grad_scale, es);
    if (train) {
      rl_grad(a.logits, a.tgt, a.rl_sample, a.rl_lse, a.rl_score, a.count, a.rl_scal, B, Lq, L.V, cfg.pad_idx, w,
              a.dlogits, act, es);
      backward(es, /*step_params=*/true);
    }
    rl_B = 0;
    leave(cs);
  }
  int rl_B = 0;
  // resident feature store: when set, forward() gathers image in_idx[b] from feats/pos
  const int32_t* in_idx = nullptr;
  int in_n_img = 0;

  // ------------------------------------------------------------------------------------
  // decoding (model.py:101-200), KV-cached.  Bit-identical to recomputing the prefix: row
  // results of every kernel are independent of how many rows/positions are in the launch.
  void encode_only(const void* feats, DType ft, const float* pos, int B, int N, hipStream_t s) {
    const int Me = B * N, d = L.d, He = L.He, dke = d / He;
    ensure_acts(B, N, 2);
    pack_encoder_input(feats, ft, pos, Me, L.F, L.P, L.Kp, a.Aenc, act, a.valid, s);
    if (L.has_img) {
      image_objects_fwd(B, N, false, s);
    } else {
      linear(a.Aenc, L.Kp, L.enc_emb_W, L.Kp, a.tmp, d, act, Me, d, L.Kp, nullptr, 0, s);
      LnFwd ln;
      ln.M = Me, ln.d = d, ln.a = a.tmp, ln.gamma = P(L.enc_lng), ln.beta = P(L.enc_lnb), ln.y = a.X[0];
      lnf(ln, s);
    }
    RowMask emask{};
    if (cfg.encode_mask) emask.valid = a.valid;
    for (int l = 0; l < L.Le; ++l) {
      const auto& w = L.enc[l];
      auto& A = a.enc[l];
      AttnGeom g;
      g.B = B, g.H = He, g.Lq = N, g.Lk = N, g.dk = dke;
      g.q = A.qkv, g.q_ld = 3 * d, g.q_bs = (int64_t)N * 3 * d;
      g.k = at(A.qkv, d), g.k_ld = 3 * d, g.k_bs = (int64_t)N * 3 * d;
      g.v = at(A.qkv, 2 * d), g.v_ld = 3 * d, g.v_bs = (int64_t)N * 3 * d;
      g.o_ld = d, g.o_bs = (int64_t)N * d;
      if (cfg.encode_mask) g.key_valid = a.valid, g.kv_bs = N, g.causal = 1;
      g.temperature = std::sqrt((float)dke);
      self_attention(a.X[l], w.Wqkv, Me, d, g, A.qkv, A.att, nullptr, s);
      linear(A.att, d, w.Wo, d, a.tmp, d, act, Me, d, d, nullptr, 0, s);
      LnFwd l1;
      l1.M = Me, l1.d = d, l1.a = a.tmp, l1.res = a.X[l], l1.gamma = P(w.ln1g), l1.beta = P(w.ln1b), l1.y = A.Y;
      lnf(l1, s);
      linear(A.Y, d, w.W1, d, A.H, L.fe, act, Me, L.fe, d, P(w.b1), 1, s);
      linear(A.H, L.fe, w.W2, L.fe, a.tmp, d, act, Me, d, L.fe, nullptr, 0, s);
      LnFwd l2;
      l2.M = Me, l2.d = d, l2.a = a.tmp, l2.a_bias = P(w.b2), l2.res = A.Y, l2.gamma = P(w.ln2g);
      l2.beta = P(w.ln2b), l2.mask = emask, l2.y = a.X[l + 1];
      lnf(l2, s);
    }
    linear(a.X[L.Le], d, L.Wkv_all, d, a.KV, (int64_t)L.Ld * 2 * L.dd, act, Me, L.Ld * 2 * L.dd, d, nullptr, 0, s);
  }

  void plan_gen(Planner& p, int R, int N) {
    const int64_t dd = L.dd, Tc = L.maxlen, e = es_();
    auto T_ = [&](void*& ptr, int64_t n) { ptr = p.raw(n * e); };
    T_(g.x, R * dd);
    T_(g.x1, R * dd);
    T_(g.x2, R * dd);
    T_(g.q, R * dd);
    T_(g.att, R * dd);
    T_(g.tmp, R * std::max<int64_t>(dd, L.dwe));
    T_(g.h, (int64_t)R * L.fd);
    T_(g.E, (int64_t)R * L.dwe);
    p.take(g.mean, R);
    p.take(g.rstd, R);
    p.take(g.Pc, (size_t)R * L.Hd * N);
    p.take(g.logits, (size_t)R * L.V);
    p.take(g.dstats, (size_t)R * ((L.V + 15) / 16));
    p.take(g.cand_v, (size_t)R * 16);
    p.take(g.cand_i, (size_t)R * 16);
    T_(g.cache, (int64_t)L.Ld * R * Tc * 2 * dd);
    p.take(g.ids, (size_t)R * Tc);
    p.take(g.ids2, (size_t)R * Tc);
    p.take(g.kvrow, (size_t)R * Tc);
    p.take(g.kvrow2, (size_t)R * Tc);
    p.take(g.seq, (size_t)R * Tc);
    p.take(g.seq2, (size_t)R * Tc);
    p.take(g.bprob, R);
    p.take(g.bprob2, R);
    p.take(g.bsrc, R);
    p.take(g.btok, R);
    p.take(g.out_ids, (size_t)R * (Tc + 1));
    p.take(g.out_attn, (size_t)(Tc - 1) * R * N);
  }
  void ensure_gen(int R, int N) {
    if (gws && R <= g.R && N <= g.N) return;
    int nR = std::max(R, g.R), nN = std::max(N, g.N);
    if (gws) {
      hz::host_sync(es);
      CAPGEN_HIP(hipFree(gws));
      gws = nullptr;
      drop_gen_graph();
    }
    Planner p;
    plan_gen(p, nR, nN);
    CAPGEN_HIP(hipMalloc(&gws, p.used));
    Planner q;
    q.base = (char*)gws;
    plan_gen(q, nR, nN);
    g.R = nR, g.N = nN;
  }

  // decoder for position t of R rows (rows r -> image r % Bimg); tokens = ids[:, t].
  // Leaves logits [R, V] in g.logits; cross-attn probs of the last block in g.Pc if want_attn.
  // bf16 decode: each decoder LayerNorm whose output feeds a register-B GEMM (the cross-query
  // projection, the FFN's first Linear, the next block's QKV projection) runs inside that GEMM
  // (GemmArgs::ln_gamma, gemm_breg.hip breg_ln_kernel): the consumer reads the producing Linear's
  // output (bias included) and the residual, normalises the rows and its column-tile-0 workgroups
  // store them as the next residual.  17 of the 19 LayerNorm launches of a token go away
  // (CAPGEN_DECODE_LN_FOLD=0: separate launches).
  // Every site below 1024 rows (greedy's 256; CAPGEN_DECODE_LN_FOLD=2: at any row count); at beam-5's
  // 1280 rows only the cross-query site: folding the QKV / FFN-up sites too replaces their 64 x 64
  // register-B tiles and measured slower (13.56-13.57 vs 12.82-12.84 ms per batch).
  int decode_ln_fold = knob(Knob::DecodeLnFold);
  // 2: every site, 1: only the cross-query site (beam's rows: 12.50-12.53 vs 12.62-12.73 ms per C4
  // batch with none, profiles/r05_decode_16row_tiles.txt), 0: none
  int ln_fold(int M) const {
    if (!decode_ln_fold || !breg_decode() || L.dd != 512 || L.fd % 64 != 0) return 0;
    for (const auto& w : L.dec)
      if (!DT(w.Wqkv) || !DT(w.Wq_c) || !DT(w.W1)) return 0;
    return decode_ln_fold == 2 || M < 1024 ? 2 : 1;
  }
  // one decode Linear: C (+)= X . W^T (+ bias) (ReLU); lng: the A rows are LayerNorm inputs, normalised
  // with (lng, lnb) and the row mask rm inside the GEMM, the normalised rows stored into lny
  void dec_linear(const void* X, int64_t woff, int M, int N, int K, void* C, const float* bias, int relu,
                  hipStream_t s, const void* lnres = nullptr, const float* lng = nullptr, const float* lnb = nullptr,
                  void* lny = nullptr, const RowMask* rm = nullptr) {
    GemmArgs ga;
    ga.M = M, ga.N = N, ga.K = K, ga.A = X, ga.lda = K, ga.B = W(woff), ga.ldb = K, ga.C = C, ga.ldc = N;
    ga.bt = DT(woff), ga.bias = bias, ga.relu = relu, ga.prio = prio(s);
    ga.ln_res = lnres, ga.ln_gamma = lng, ga.ln_beta = lnb, ga.ln_y = lny;
    if (rm) ga.ln_ids = rm->ids, ga.ln_ids_ld = rm->ids_ld, ga.ln_pad = rm->pad_idx;
    if (stamp_on) ga.stamp = stamp(s, std::string(lng ? "gemm fwd+ln " : "gemm fwd ") + dims(M, N, K));
    gemm(ga, act, act, false, false, s);
  }

  void dec_step(int R, int Bimg, int N, int t, void* cache, const int32_t* ids, bool want_attn, hipStream_t s,
                const int32_t* kv_row = nullptr) {
    const int dd = L.dd, Hd = L.Hd, dkd = dd / Hd, Tc = L.maxlen;
    GemmArgs ge;  // the embedding rows gathered by the projection GEMM itself (where it takes the shape)
    ge.M = R, ge.N = dd, ge.K = L.dwe, ge.A = emb_bf, ge.lda = L.dwe, ge.B = W(L.Wel), ge.ldb = L.dwe;
    ge.C = g.tmp, ge.ldc = dd, ge.bt = DT(L.Wel), ge.prio = prio(s);
    ge.a_ids = ids + t, ge.a_ids_ld = Tc, ge.a_table_rows = L.V;
    if (emb_bf && ge.bt && gemm_breg_ok(ge)) {
      if (stamp_on) ge.stamp = stamp(s, "gemm fwd (gathered A) " + dims(R, dd, L.dwe));
      gemm(ge, act, act, false, false, s);
    } else {
      embedding_gather(P(L.emb), ids + t, Tc, R, L.dwe, g.E, act, s, L.V);
      linear(g.E, L.dwe, L.Wel, L.dwe, g.tmp, dd, act, R, dd, L.dwe, nullptr, 0, s, DT(L.Wel));
    }
    LnFwd ln;
    ln.M = R, ln.d = dd, ln.a = g.tmp, ln.pe = pe + (int64_t)t * dd, ln.pe_L = 1, ln.gamma = P(L.dec_lng);
    ln.beta = P(L.dec_lnb), ln.y = g.x;
    lnf(ln, s);
    RowMask rm{};
    rm.ids = ids + t, rm.ids_ld = Tc, rm.pad_idx = cfg.pad_idx;
    const int64_t kvld = (int64_t)L.Ld * 2 * dd, cld = (int64_t)Tc * 2 * dd;
    const int fmode = ln_fold(R);
    const bool fold = fmode == 2, fold1 = fmode >= 1;  // every site / the cross-query site
    for (int l = 0; l < L.Ld; ++l) {
      const auto& w = L.dec[l];
      void* cl = at(cache, (int64_t)l * R * cld);
      if (act == DType::BF16) {  // one GEMM: Q columns -> g.q, K/V columns -> the cache at position t
        GemmArgs ga;
        ga.M = R, ga.N = 3 * dd, ga.K = dd, ga.A = g.x, ga.lda = dd, ga.B = W(w.Wqkv), ga.ldb = dd;
        ga.C = g.q, ga.ldc = dd, ga.C2 = at(cl, (int64_t)t * 2 * dd), ga.ldc2 = cld, ga.nsplit = dd;
        ga.bt = DT(w.Wqkv);
        if (fold && l > 0) {  // the previous block's FFN LayerNorm (W2 output in tmp + x2) -> g.x
          const auto& wp = L.dec[l - 1];
          ga.A = g.tmp, ga.ln_res = g.x2, ga.ln_gamma = P(wp.lfg), ga.ln_beta = P(wp.lfb), ga.ln_y = g.x;
          ga.ln_ids = rm.ids, ga.ln_ids_ld = rm.ids_ld, ga.ln_pad = rm.pad_idx;
        }
        ga.prio = prio(s);
        if (stamp_on) ga.stamp = stamp(s, std::string(ga.ln_gamma ? "gemm fwd+ln " : "gemm fwd ") + dims(R, 3 * dd, dd));
        gemm(ga, act, act, false, false, s);
      } else {
        linear(g.x, dd, w.Wqkv, dd, g.q, dd, act, R, dd, dd, nullptr, 0, s);
        linear(g.x, dd, w.Wqkv + (int64_t)dd * dd, dd, at(cl, (int64_t)t * 2 * dd), cld, act, R, 2 * dd, dd, nullptr,
               0, s);
      }
      AttnGeom sg;
      sg.B = R, sg.H = Hd, sg.Lq = 1, sg.Lk = t + 1, sg.dk = dkd;
      sg.q = g.q, sg.q_ld = dd, sg.q_bs = dd;
      sg.k = cl, sg.k_ld = 2 * dd, sg.k_bs = cld;
      sg.v = at(cl, dd), sg.v_ld = 2 * dd, sg.v_bs = cld;
      sg.o_ld = dd, sg.o_bs = dd;
      sg.key_ids = ids, sg.kid_bs = Tc, sg.pad_idx = cfg.pad_idx, sg.causal = 1, sg.q_pos0 = t;
      sg.kv_row = kv_row, sg.kv_row_ld = Tc;
      sg.temperature = std::sqrt((float)dkd);
      attf(sg, g.att, nullptr, act, s);
      if (fold1) {  // att . Wo_s^T into tmp; the cross-query GEMM normalises tmp + x (-> g.x1)
        dec_linear(g.att, w.Wo_s, R, dd, dd, g.tmp, nullptr, 0, s);
        dec_linear(g.tmp, w.Wq_c, R, dd, dd, g.q, nullptr, 0, s, g.x, P(w.lsg), P(w.lsb), g.x1);
      } else {
        linear(g.att, dd, w.Wo_s, dd, g.tmp, dd, act, R, dd, dd, nullptr, 0, s, DT(w.Wo_s));
        LnFwd l1;
        l1.M = R, l1.d = dd, l1.a = g.tmp, l1.res = g.x, l1.gamma = P(w.lsg), l1.beta = P(w.lsb), l1.y = g.x1;
        lnf(l1, s);
        linear(g.x1, dd, w.Wq_c, dd, g.q, dd, act, R, dd, dd, nullptr, 0, s, DT(w.Wq_c));
      }
      const bool want_p = want_attn && l == L.Ld - 1;
      AttnGeom c;  // rows r -> image r % Bimg
      c.H = Hd, c.Lk = N, c.dk = dkd;
      c.k = at(a.KV, (int64_t)l * 2 * dd), c.k_ld = kvld, c.k_bs = (int64_t)N * kvld;
      c.v = at(a.KV, (int64_t)l * 2 * dd + dd), c.v_ld = kvld, c.v_bs = (int64_t)N * kvld;
      c.key_valid = a.valid, c.kv_bs = N;
      c.temperature = std::sqrt((float)dkd);
      const int kb = R / Bimg;  // beam rows per image: row j * Bimg + b
      if (act == DType::BF16 && cross_mfma_on && !want_p && kb > 1 && R % Bimg == 0 && kb <= 64) {
        // an image's kb beam rows as ONE query block of the MFMA attention (attention_mfma.hip), one
        // workgroup per (image, head): the rows are Bimg * d apart
        c.B = Bimg, c.Lq = kb;
        c.q = g.q, c.q_ld = (int64_t)Bimg * dd, c.q_bs = dd;
        c.o_ld = (int64_t)Bimg * dd, c.o_bs = dd;
      } else {
        c.B = R, c.Lq = 1;
        c.q = g.q, c.q_ld = dd, c.q_bs = dd;
        c.kv_bmod = Bimg;
        c.o_ld = dd, c.o_bs = dd;
      }
      attf(c, g.att, want_p ? g.Pc : nullptr, act, s);
      if (fold) {  // att . Wo_c^T into tmp, the FFN's first GEMM normalises tmp + x1 (-> g.x2);
                   // h . W2^T + b2 into tmp, normalised with x2 by the next block's QKV GEMM
        dec_linear(g.att, w.Wo_c, R, dd, dd, g.tmp, nullptr, 0, s);
        dec_linear(g.tmp, w.W1, R, L.fd, dd, g.h, P(w.b1), 1, s, g.x1, P(w.lcg), P(w.lcb), g.x2);
        dec_linear(g.h, w.W2, R, dd, L.fd, g.tmp, P(w.b2), 0, s);
        if (l == L.Ld - 1) {  // the last block's FFN LayerNorm feeds the classifier: its own launch
          LnFwd l3;
          l3.M = R, l3.d = dd, l3.a = g.tmp, l3.res = g.x2, l3.gamma = P(w.lfg), l3.beta = P(w.lfb);
          l3.mask = rm, l3.y = g.x;
          lnf(l3, s);
        }
        continue;
      }
      linear(g.att, dd, w.Wo_c, dd, g.tmp, dd, act, R, dd, dd, nullptr, 0, s, DT(w.Wo_c));
      LnFwd l2;
      l2.M = R, l2.d = dd, l2.a = g.tmp, l2.res = g.x1, l2.gamma = P(w.lcg), l2.beta = P(w.lcb), l2.y = g.x2;
      lnf(l2, s);
      linear(g.x2, dd, w.W1, dd, g.h, L.fd, act, R, L.fd, dd, P(w.b1), 1, s, DT(w.W1));
      linear(g.h, L.fd, w.W2, L.fd, g.tmp, dd, act, R, dd, L.fd, nullptr, 0, s, DT(w.W2));
      LnFwd l3;
      l3.M = R, l3.d = dd, l3.a = g.tmp, l3.a_bias = P(w.b2), l3.res = g.x2, l3.gamma = P(w.lfg), l3.beta = P(w.lfb);
      l3.mask = rm, l3.y = g.x;
      lnf(l3, s);
    }
    const void* xo = g.x;
    if (L.has_mf) {  // rows r -> image r % Bimg
      move_first_fwd(g.x, a.X[L.Le], R, 1, Bimg, N, g.x2, g.h, g.tmp, g.x1, nullptr, nullptr, nullptr, false, s);
      xo = g.x1;
    }
    if (slab_decode()) {  // f32 logits + per-16-column-slab {max, exp-sum} for the selection
      GemmArgs ga;
      ga.M = R, ga.N = L.V, ga.K = dd, ga.A = xo, ga.lda = dd, ga.B = W(L.Wc), ga.ldb = dd;
      ga.C = g.logits, ga.ldc = L.V, ga.bias = P(L.bc);
      ga.dec_stats = g.dstats, ga.dec_ld = (L.V + 15) / 16;
      if (stamp_on) ga.stamp = stamp(s, "gemm NT " + dims(R, L.V, dd) + " classifier+slab stats");
      gemm(ga, act, DType::F32, false, false, s);
    } else {
      linear(xo, dd, L.Wc, dd, g.logits, L.V, DType::F32, R, L.V, dd, P(L.bc), 0, s);
    }
  }
  // bf16 beam decode: the cross attention of an image's beam rows on the MFMA attention kernel
  // (CAPGEN_DECODE_CROSS_MFMA=0: the grouped VALU decode kernel, attention.hip)
  bool cross_mfma_on = knob(Knob::DecodeCrossMfma) != 0;
  bool fused_beam_step_on = knob(Knob::FusedBeamStep) != 0;
  // bf16 decode: the classifier epilogue writes slab stats and the greedy / beam selection reads
  // k * 16 logits per row instead of the whole row (CAPGEN_SLAB_DECODE=0: full-row kernels)
  bool slab_decode_on = knob(Knob::SlabDecode) != 0;
  bool slab_decode() const { return slab_decode_on && act == DType::BF16 && L.V % 4 == 0 && slab_select_ok(L.V); }

  void greedy(const void* feats, DType ft, const float* pos, int B, int N, int64_t* ids_out, float* attn_out,
              hipStream_t s) {
    require(N >= 1 && N <= 64, "greedy: N must be in [1, 64]");
    require(B >= 1, "greedy: need B >= 1");
    ensure_acts(B, N, 2);
    ensure_gen(B, N);
    ensure_dtiles();
    const GenKey key{(attn_out ? 1 : 0) + (decode_logsm ? 8 : 0), feats, pos, (int)ft, B, N, 0};
    gen_run(key, [&] { greedy_body(feats, ft, pos, B, N, g.out_ids, attn_out ? g.out_attn : nullptr, s); }, s);
    CAPGEN_HIP(hipMemcpyAsync(ids_out, g.out_ids, sizeof(int64_t) * B * (L.maxlen + 1), hipMemcpyDeviceToDevice, s));
    if (attn_out)
      CAPGEN_HIP(hipMemcpyAsync(attn_out, g.out_attn, sizeof(float) * (L.maxlen - 1) * B * N, hipMemcpyDeviceToDevice,
                                s));
  }
  void greedy_body(const void* feats, DType ft, const float* pos, int B, int N, int64_t* ids_out, float* attn_out,
                   hipStream_t s) {
    encode_only(feats, ft, pos, B, N, s);
    ensure_gen(B, N);
    build_dtiles(s);
    const int Tc = L.maxlen, W = L.maxlen + 1;
    init_gen_ids_kernel<<<(B * std::max(W, Tc) + 255) / 256, 256, 0, s>>>(ids_out, B, W, g.ids, Tc);
    CAPGEN_HIP(hipGetLastError());
    for (int t = 0; t < L.maxlen - 1; ++t) {
      dec_step(B, B, N, t, g.cache, g.ids, attn_out != nullptr, s);
      if (attn_out) attention_head_mean(g.Pc, B, L.Hd, 1, N, 0, attn_out + (int64_t)t * B * N, s);
      if (slab_decode())  // argmax of the logits = argmax of the (log-)softmax
        slab_argmax(g.logits, g.dstats, B, L.V, ids_out, W, t + 1, g.ids + t + 1, Tc, s);
      else
        argmax_softmax(g.logits, B, L.V, ids_out, W, t + 1, g.ids + t + 1, Tc, s, decode_logsm);
    }
  }

  void beam(const void* feats, DType ft, const float* pos, int B, int N, int k, int64_t* ids_out, hipStream_t s) {
    require(k >= 1 && k <= 16, "beam_search: beam_size must be in [1, 16]");
    require(k <= L.V, "beam_search: beam_size must be <= num_vocab");
    require(B >= 1 && N >= 1 && N <= 64, "beam_search: need B >= 1 and N in [1, 64]");
    ensure_acts(B, N, 2);
    ensure_gen(k * B, N);
    ensure_dtiles();
    const GenKey key{2 + (decode_logsm ? 8 : 0), feats, pos, (int)ft, B, N, k};
    gen_run(key, [&] { beam_body(feats, ft, pos, B, N, k, g.out_ids, s); }, s);
    CAPGEN_HIP(hipMemcpyAsync(ids_out, g.out_ids, sizeof(int64_t) * B * L.maxlen, hipMemcpyDeviceToDevice, s));
  }
  void beam_body(const void* feats, DType ft, const float* pos, int B, int N, int k, int64_t* ids_out, hipStream_t s) {
    const int R = k * B, Tc = L.maxlen, Tw = L.maxlen, dd = L.dd;
    encode_only(feats, ft, pos, B, N, s);
    ensure_gen(R, N);
    build_dtiles(s);
    init_gen_ids_kernel<<<(R * Tc + 255) / 256, 256, 0, s>>>(g.seq, R, Tw, g.ids, Tc);
    CAPGEN_HIP(hipGetLastError());
    // position 0: every beam holds <START>; top-k of beam 0's distribution (model.py:148-166)
    beam_kvrow_kernel<<<(R * Tc + 255) / 256, 256, 0, s>>>(g.kvrow2, g.kvrow, Tc, -1, g.ids, B, R);  // [r][0] = r
    dec_step(R, B, N, 0, g.cache, g.ids, false, s);
    // bf16: the selection and the reorder of a step as one launch per image (beam_slab_step:
    // CAPGEN_FUSED_BEAM_STEP=0 restores the top-k, merge and three reorder launches)
    const bool fused_step = slab_decode() && fused_beam_step_on && k <= 16 && Tw == Tc;
    auto fused = [&](int t, const float* prev, int kin, float* out_prob) {
      beam_slab_step(g.logits, g.dstats, prev, kin, B, L.V, k, decode_logsm, out_prob, g.bsrc, g.btok, g.seq, g.seq2,
                     Tw, g.ids, g.ids2, g.kvrow, g.kvrow2, Tc, t, s);
      std::swap(g.seq, g.seq2);
      std::swap(g.ids, g.ids2);
      std::swap(g.kvrow, g.kvrow2);
    };
    if (fused_step)  // (beam 0's finalists only: every source is beam 0 at t = 0)
      fused(0, nullptr, 1, g.bprob);
    else if (slab_decode())
      beam_step_topk_slab(g.logits, g.dstats, nullptr, 1, B, L.V, k, decode_logsm, g.cand_v, g.cand_i, g.bprob, g.bsrc,
                          g.btok, s);
    else
      beam_step_topk(g.logits, nullptr, 1, B, L.V, k, decode_logsm, g.cand_v, g.cand_i, g.bprob, g.bsrc, g.btok, s);
    if (!fused_step) CAPGEN_HIP(hipMemsetAsync(g.bsrc, 0, sizeof(int32_t) * R, s));  // all beams descend from beam 0
    // The K/V cache is never copied: row r writes its position-t K/V at [l][r][t] and reads
    // position j of its history from row kvrow[r][j] (the beam it descended from there); a
    // reorder moves only the ids / sequences and this [R][Tc] table
    auto reorder = [&](int t) {
      // seq/ids rows follow their source beam, then column t+1 = chosen token
      dim3 gs(1, R);
      beam_gather_kernel<int64_t><<<gs, 64, 0, s>>>(g.seq, g.seq2, Tw, Tw, g.bsrc, B, R, g.btok, t + 1);
      beam_gather_kernel<int32_t><<<gs, 64, 0, s>>>(g.ids, g.ids2, Tc, Tc, g.bsrc, B, R, g.btok, t + 1);
      beam_kvrow_kernel<<<(R * Tc + 255) / 256, 256, 0, s>>>(g.kvrow, g.kvrow2, Tc, t, g.bsrc, B, R);
      CAPGEN_HIP(hipGetLastError());
      std::swap(g.seq, g.seq2);
      std::swap(g.ids, g.ids2);
      std::swap(g.kvrow, g.kvrow2);
    };
    if (!fused_step) reorder(0);
    for (int t = 1; t < Tw - 1; ++t) {
      dec_step(R, B, N, t, g.cache, g.ids, false, s, g.kvrow);
      if (fused_step) {
        fused(t, g.bprob, k, g.bprob2);
        std::swap(g.bprob, g.bprob2);
        continue;
      }
      if (slab_decode())
        beam_step_topk_slab(g.logits, g.dstats, g.bprob, k, B, L.V, k, decode_logsm, g.cand_v, g.cand_i, g.bprob2,
                            g.bsrc, g.btok, s);
      else
        beam_step_topk(g.logits, g.bprob, k, B, L.V, k, decode_logsm, g.cand_v, g.cand_i, g.bprob2, g.bsrc, g.btok,
                       s);
      std::swap(g.bprob, g.bprob2);
      reorder(t);
    }
    CAPGEN_HIP(hipMemcpyAsync(ids_out, g.seq, sizeof(int64_t) * B * Tw, hipMemcpyDeviceToDevice, s));
  }

  ~capgen_engine() {
    if (es) (void)hipStreamSynchronize(es);
    drop_graph();
    if (comm) ncclCommDestroy(comm);
    for (void* p : {(void*)params, (void*)grads, (void*)am, (void*)av, (void*)shadow, (void*)wtile, (void*)dtiles, (void*)emb_bf, (void*)pe, (void*)step,
                    (void*)adam_scal, (void*)seed, (void*)scalars, (void*)gstripe, ws, gws, (void*)stamp_ring})
      if (p) (void)hipFree(p);
    if (count_host) (void)hipHostFree(count_host);
    if (dp_chk) (void)hipFree(dp_chk);
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_out) (void)hipEventDestroy(ev_out);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    for (hipEvent_t e : {ev_b1, ev_b2, ev_cj, ev_count, ev_ff, ev_fj})
      if (e) (void)hipEventDestroy(e);
    if (ec && ec != es && ec != es2) (void)hipStreamSynchronize(ec), (void)hipStreamDestroy(ec);
    if (es2 && es2 != es) (void)hipStreamSynchronize(es2), (void)hipStreamDestroy(es2);
    if (es) (void)hipStreamDestroy(es);
  }
};

// =========================================================================================
// C ABI
// =========================================================================================
namespace capgen {
void scst_rewards(const int64_t* target, int64_t target_ld, const int64_t* sample, int64_t sample_ld, int B, int L,
                  int start_id, int end_id, int null_id, int64_t dot_id, double cider_w, double bleu_w, double* out);
}

namespace {

template <class F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const Error& e) {
    g_last_error = e.msg;
  } catch (const std::exception& e) {
    g_last_error = e.what();
  } catch (...) {
    g_last_error = "unknown error";
  }
  return 1;
}

DType dt(int x) {
  require(x == CAPGEN_F32 || x == CAPGEN_BF16, "dtype must be CAPGEN_F32 or CAPGEN_BF16");
  return x == CAPGEN_F32 ? DType::F32 : DType::BF16;
}

void set_device(capgen_t* h) {
  require(h != nullptr, "null engine handle");
  CAPGEN_HIP(hipSetDevice(h->device));
}

void pe_table(const Layout& L, std::vector<float>& out) {
  // model.py:502-514: float64 angles, sin on even columns, cos on odd, cast to f32
  const int n = L.maxlen - 1, d = L.dd;
  out.resize((size_t)n * d);
  for (int p = 0; p < n; ++p)
    for (int j = 0; j < d; ++j) {
      double ang = (double)p / std::pow(10000.0, 2.0 * (j / 2) / (double)d);
      out[(size_t)p * d + j] = (float)((j % 2 == 0) ? std::sin(ang) : std::cos(ang));
    }
}

}  // namespace

extern "C" {

const char* capgen_last_error(void) { return g_last_error.c_str(); }
int capgen_abi_version(void) { return CAPGEN_ABI_VERSION; }

int capgen_set_knob(const char* name, int value, int* old) {
  return guarded([&] {
    require(name != nullptr, "set_knob: null name");
    const int rc = knob_set(name, value, old);
    require(rc != -1, std::string("set_knob: unknown switch ") + name);
    require(rc != -2, std::string("set_knob: ") + name + " exists only in the debug build (libcapgen_debug.so)");
  });
}

int capgen_debug_build(void) { return debug_build() ? 1 : 0; }

int capgen_param_table(const capgen_config* cfg, capgen_param_info* out, int cap, int* count, int64_t* arena_elems) {
  return guarded([&] {
    require(cfg != nullptr, "null config");
    Layout L = make_layout(*cfg);
    if (count) *count = (int)L.table.size();
    if (arena_elems) *arena_elems = L.total;
    for (int i = 0; i < (int)L.table.size() && i < cap && out; ++i) out[i] = L.table[i];
  });
}

int capgen_create(const capgen_config* cfg, int device, capgen_t** out) {
  return guarded([&] {
    require(cfg && out, "null argument");
    *out = nullptr;
    int ndev = 0;
    CAPGEN_HIP(hipGetDeviceCount(&ndev));
    require(device >= 0 && device < ndev, "capgen_create: invalid device index");
    CAPGEN_HIP(hipSetDevice(device));
    gemm_init();
    auto h = std::make_unique<capgen_engine>();
    h->cfg = *cfg;
    h->L = make_layout(*cfg);
    h->device = device;
    h->act = dt(cfg->dtype);
    const size_t n = (size_t)h->L.total;
    // (stream priorities measured: no gain for one engine, and with two engines in a process
    // the high-priority queues serialised each other -- plain streams)
    CAPGEN_HIP(hipStreamCreateWithFlags(&h->es, hipStreamNonBlocking));
    // CAPGEN_STREAMS (experiment knob): 3 = critical path + weight-grad + bucket streams
    // (default), 2 = buckets on the weight-grad stream, 1 = everything on one stream
    const int nstreams = knob(Knob::Streams);
    if (nstreams >= 2) CAPGEN_HIP(hipStreamCreateWithFlags(&h->es2, hipStreamNonBlocking));
    else h->es2 = h->es;
    // the fork / join / bucket events only order this device's own streams, so they skip the
    // system-scope acquire / release HIP puts on an event by default (that fence writes back and
    // invalidates L2 around every record / wait; the kernels' own device-scope fences order the
    // streams).  Measured, three alternating runs each: 2.760-2.776 ms/step vs 2.817-2.838 with the
    // system fence, 2.815-2.832 with a device-scope release only (CAPGEN_EVENT_FENCE = 1 / 0 / 2).
    const int ef = knob(Knob::EventFence);
    const unsigned evf = hipEventDisableTiming | (ef == 1 ? hipEventDisableSystemFence : ef == 2 ? hipEventReleaseToDevice : 0u);
    CAPGEN_HIP(hipEventCreateWithFlags(&h->ev_fork, evf));
    CAPGEN_HIP(hipEventCreateWithFlags(&h->ev_join, evf));
    if (nstreams >= 3) CAPGEN_HIP(hipStreamCreateWithFlags(&h->ec, hipStreamNonBlocking));
    else h->ec = h->es2;
    for (hipEvent_t* e : {&h->ev_b1, &h->ev_b2, &h->ev_cj, &h->ev_ff, &h->ev_fj})
      CAPGEN_HIP(hipEventCreateWithFlags(e, evf));
    CAPGEN_HIP(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
    CAPGEN_HIP(hipEventCreateWithFlags(&h->ev_count, hipEventDisableTiming));
    CAPGEN_HIP(hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming));
    CAPGEN_HIP(hipMalloc(&h->params, n * 4));
    CAPGEN_HIP(hipMalloc(&h->grads, n * 4));
    CAPGEN_HIP(hipMalloc(&h->am, n * 4));
    CAPGEN_HIP(hipMalloc(&h->av, n * 4));
    CAPGEN_HIP(hipMemset(h->params, 0, n * 4));
    CAPGEN_HIP(hipMemset(h->grads, 0, n * 4));
    CAPGEN_HIP(hipMemset(h->am, 0, n * 4));
    CAPGEN_HIP(hipMemset(h->av, 0, n * 4));
    if (h->act == DType::BF16) {
      CAPGEN_HIP(hipMalloc(&h->shadow, (size_t)h->L.n_dense * 2));
      CAPGEN_HIP(hipMemset(h->shadow, 0, (size_t)h->L.n_dense * 2));
      h->build_tiles();
    }
    std::vector<float> pe;
    pe_table(h->L, pe);
    CAPGEN_HIP(hipMalloc(&h->pe, pe.size() * 4));
    CAPGEN_HIP(hipMemcpy(h->pe, pe.data(), pe.size() * 4, hipMemcpyHostToDevice));
    CAPGEN_HIP(hipMalloc(&h->step, 64));
    CAPGEN_HIP(hipMemset(h->step, 0, 64));
    CAPGEN_HIP(hipMalloc(&h->adam_scal, 64));
    CAPGEN_HIP(hipMalloc(&h->seed, 64));
    uint64_t sd = cfg->seed;
    CAPGEN_HIP(hipMemcpy(h->seed, &sd, 8, hipMemcpyHostToDevice));
    CAPGEN_HIP(hipMalloc(&h->scalars, 256));
    h->n_small = h->L.total - h->L.enc_lng;
    CAPGEN_HIP(hipMalloc(&h->gstripe, (size_t)capgen_engine::NSTRIPE * h->n_small * sizeof(float)));
    CAPGEN_HIP(hipHostMalloc(&h->count_host, 64, hipHostMallocDefault));
    // the null-stream memsets above are not ordered before the engine's non-blocking streams
    hz::host_sync(nullptr);
    *out = h.release();
  });
}

int capgen_destroy(capgen_t* h) {
  return guarded([&] {
    if (!h) return;
    (void)hipSetDevice(h->device);
    delete h;
  });
}

int capgen_get_params(capgen_t* h, float* dst, int64_t n) {
  return guarded([&] {
    set_device(h);
    require(n == h->L.total, "get_params: size mismatch");
    hz::host_sync(h->es);
    CAPGEN_HIP(hipMemcpy(dst, h->params, n * 4, hipMemcpyDeviceToHost));
  });
}

int capgen_set_params(capgen_t* h, const float* src, int64_t n) {
  return guarded([&] {
    set_device(h);
    require(n == h->L.total, "set_params: size mismatch");
    hz::host_sync(h->es);
    CAPGEN_HIP(hipMemcpy(h->params, src, n * 4, hipMemcpyHostToDevice));
    h->refresh_shadow(h->es);
    hz::host_sync(h->es);
  });
}

int capgen_get_grads(capgen_t* h, float* dst, int64_t n) {
  return guarded([&] {
    set_device(h);
    require(n == h->L.total, "get_grads: size mismatch");
    require(!h->grads_sharded, "get_grads: after a sharded (ZeRO-1) step the gradient arena holds this rank's "
                               "reduce-scattered chunks only (CAPGEN_ZERO=0 keeps whole gradients)");
    hz::host_sync(h->es);
    CAPGEN_HIP(hipMemcpy(dst, h->grads, n * 4, hipMemcpyDeviceToHost));
  });
}

int capgen_set_grads(capgen_t* h, const float* src, int64_t n) {
  return guarded([&] {
    set_device(h);
    require(n == h->L.total, "set_grads: size mismatch");
    hz::host_sync(h->es);
    CAPGEN_HIP(hipMemcpy(h->grads, src, n * 4, hipMemcpyHostToDevice));
  });
}

int capgen_get_adam_state(capgen_t* h, int64_t* step, float* m, float* v, int64_t n) {
  return guarded([&] {
    set_device(h);
    require(n == h->L.total, "get_adam_state: size mismatch");
    require(!h->moments_sharded, "get_adam_state: the moments are sharded across ranks (ZeRO-1): call "
                                 "capgen_dp_sync_adam_state on every rank first");
    hz::host_sync(h->es);
    if (step) CAPGEN_HIP(hipMemcpy(step, h->step, 8, hipMemcpyDeviceToHost));
    if (m) CAPGEN_HIP(hipMemcpy(m, h->am, n * 4, hipMemcpyDeviceToHost));
    if (v) CAPGEN_HIP(hipMemcpy(v, h->av, n * 4, hipMemcpyDeviceToHost));
  });
}

int capgen_set_adam_state(capgen_t* h, int64_t step, const float* m, const float* v, int64_t n) {
  return guarded([&] {
    set_device(h);
    require(n == h->L.total, "set_adam_state: size mismatch");
    hz::host_sync(h->es);
    CAPGEN_HIP(hipMemcpy(h->step, &step, 8, hipMemcpyHostToDevice));
    if (m) CAPGEN_HIP(hipMemcpy(h->am, m, n * 4, hipMemcpyHostToDevice));
    else CAPGEN_HIP(hipMemset(h->am, 0, n * 4));
    if (v) CAPGEN_HIP(hipMemcpy(h->av, v, n * 4, hipMemcpyHostToDevice));
    else CAPGEN_HIP(hipMemset(h->av, 0, n * 4));
    hz::host_sync(nullptr);
  });
}

int capgen_arenas(capgen_t* h, float** params, float** grads, int64_t* n) {
  return guarded([&] {
    require(h != nullptr, "null engine handle");
    if (params) *params = h->params;
    if (grads) *grads = h->grads;
    if (n) *n = h->L.total;
  });
}

int capgen_set_training(capgen_t* h, int training) {
  return guarded([&] {
    require(h != nullptr, "null engine handle");
    h->training = training != 0;
  });
}

int capgen_set_decode_log_softmax(capgen_t* h, int enable) {
  return guarded([&] {
    require(h != nullptr, "null engine handle");
    h->decode_logsm = enable != 0;
  });
}

int capgen_set_graph(capgen_t* h, int enable) {
  return guarded([&] {
    require(h != nullptr, "null engine handle");
    h->graph_on = enable != 0;
    if (!h->graph_on) h->drop_graph();
  });
}

int capgen_forward(capgen_t* h, const void* feats, int ft, const float* pos, const int32_t* caps, int B, int N, int T,
                   float* loss_out, void* stream) {
  return guarded([&] {
    set_device(h);
    hipStream_t cs = (hipStream_t)stream;
    h->ensure_acts(B, N, T);
    h->enter(cs);
    h->forward(feats, dt(ft), pos, caps, B, N, T, loss_out, h->training, h->es);
    h->leave(cs);
  });
}

int capgen_backward(capgen_t* h, void* stream) {
  return guarded([&] {
    set_device(h);
    hipStream_t cs = (hipStream_t)stream;
    h->enter(cs);
    h->backward(h->es);
    h->allreduce_grads(h->es);
    h->leave(cs);
  });
}

int capgen_adam_step(capgen_t* h, void* stream) {
  return guarded([&] {
    set_device(h);
    hipStream_t cs = (hipStream_t)stream;
    h->enter(cs);
    h->adam(h->es);
    h->leave(cs);
  });
}

int capgen_train_step(capgen_t* h, const void* feats, int ft, const float* pos, const int32_t* caps, int B, int N,
                      int T, float* loss_out, void* stream) {
  return guarded([&] {
    set_device(h);
    h->train_step(feats, dt(ft), pos, caps, B, N, T, loss_out, (hipStream_t)stream);
    h->dp_check((hipStream_t)stream, loss_out);
  });
}

int capgen_compute_loss(capgen_t* h, const void* feats, int ft, const float* pos, const int32_t* caps, int B, int N,
                        int T, float* loss_out, void* stream) {
  // torch.no_grad() only: dropout follows the module's train/eval state (models.py:131-135)
  return capgen_forward(h, feats, ft, pos, caps, B, N, T, loss_out, stream);
}

int capgen_copy_logits(capgen_t* h, float* dst, int64_t n, void* stream) {
  return guarded([&] {
    set_device(h);
    require(h->fB > 0, "copy_logits: no forward yet");
    const int64_t want = (int64_t)h->fB * (h->fT - 1) * h->L.V;
    require(n == want, "copy_logits: size mismatch");
    hipStream_t cs = (hipStream_t)stream;
    h->enter(cs);
    if (h->fused_ce())  // the fused step never writes the logits: recompute them (test hook)
      h->linear(h->dec_out(), h->L.dd, h->L.Wc, h->L.dd, h->a.logits, h->L.V, DType::F32, h->fB * (h->fT - 1),
                h->L.V, h->L.dd, h->P(h->L.bc), 0, h->es);
    CAPGEN_HIP(hipMemcpyAsync(dst, h->a.logits, n * 4, hipMemcpyDeviceToDevice, h->es));
    h->leave(cs);
  });
}

int capgen_greedy(capgen_t* h, const void* feats, int ft, const float* pos, int B, int N, int64_t* ids_out,
                  float* attn_out, void* stream) {
  return guarded([&] {
    set_device(h);
    hipStream_t cs = (hipStream_t)stream;
    h->enter(cs);
    h->greedy(feats, dt(ft), pos, B, N, ids_out, attn_out, h->es);
    h->leave(cs);
  });
}

int capgen_beam(capgen_t* h, const void* feats, int ft, const float* pos, int B, int N, int k, int64_t* ids_out,
                void* stream) {
  return guarded([&] {
    set_device(h);
    hipStream_t cs = (hipStream_t)stream;
    h->enter(cs);
    h->beam(feats, dt(ft), pos, B, N, k, ids_out, h->es);
    h->leave(cs);
  });
}

int capgen_set_rng_seed(capgen_t* h, uint64_t sd) {
  return guarded([&] {
    set_device(h);
    hz::host_sync(h->es);
    CAPGEN_HIP(hipMemcpy(h->seed, &sd, 8, hipMemcpyHostToDevice));
  });
}

int capgen_debug_gemm(int M, int N, int K, const void* A, int64_t lda, int ta, const void* B, int64_t ldb, int tb,
                      void* Cp, int64_t ldc, int in_dtype, int out_dtype, const float* bias, float alpha, int beta,
                      int relu, void* stream) {
  return guarded([&] {
    gemm_init();
    GemmArgs ga;
    ga.M = M, ga.N = N, ga.K = K, ga.A = A, ga.lda = lda, ga.B = B, ga.ldb = ldb, ga.C = Cp, ga.ldc = ldc;
    ga.bias = bias, ga.alpha = alpha, ga.beta = beta, ga.relu = relu;
    gemm(ga, dt(in_dtype), dt(out_dtype), ta != 0, tb != 0, (hipStream_t)stream);
  });
}

int capgen_debug_gemm_tiled(int M, int N, int K, const void* A, int64_t lda, const void* B, int64_t ldb, int tb,
                            void* Bt, void* Cp, int64_t ldc, int out_dtype, const float* bias, int beta, int relu,
                            const void* aux, int64_t ldaux, void* stream) {
  return guarded([&] {
    gemm_init();
    const hipStream_t s = (hipStream_t)stream;
    gemm_tile_b(reinterpret_cast<const bf16*>(B), ldb, tb, N, K, reinterpret_cast<bf16*>(Bt), s);
    GemmArgs ga;
    ga.M = M, ga.N = N, ga.K = K, ga.A = A, ga.lda = lda, ga.B = B, ga.ldb = ldb, ga.C = Cp, ga.ldc = ldc;
    ga.bias = bias, ga.beta = beta, ga.relu = relu, ga.aux = aux, ga.ldaux = ldaux, ga.bt = Bt;
    require(gemm_breg_ok(ga), "debug_gemm_tiled: a shape / epilogue the register-B kernel does not take");
    gemm(ga, DType::BF16, dt(out_dtype), false, tb != 0, s);
  });
}

int capgen_debug_gemm_tiled_ln(int M, int N, const void* A, const void* ln_res, const void* B, void* Bt, void* Cp,
                               int out_dtype, const float* bias, int beta, int relu, const float* ln_gamma,
                               const float* ln_beta, void* ln_y, const int32_t* ln_ids, int64_t ln_ids_ld, int ln_pad,
                               void* stream) {
  return guarded([&] {
    gemm_init();
    const hipStream_t s = (hipStream_t)stream;
    const int K = 512;
    gemm_tile_b(reinterpret_cast<const bf16*>(B), K, 0, N, K, reinterpret_cast<bf16*>(Bt), s);
    GemmArgs ga;
    ga.M = M, ga.N = N, ga.K = K, ga.A = A, ga.lda = K, ga.B = B, ga.ldb = K, ga.C = Cp, ga.ldc = N;
    ga.bias = bias, ga.beta = beta, ga.relu = relu, ga.bt = Bt;
    ga.ln_res = ln_res, ga.ln_gamma = ln_gamma, ga.ln_beta = ln_beta, ga.ln_y = ln_y;
    ga.ln_ids = ln_ids, ga.ln_ids_ld = ln_ids_ld, ga.ln_pad = ln_pad;
    require(ln_gamma && gemm_breg_ok(ga), "debug_gemm_tiled_ln: a shape the folded-LayerNorm kernel does not take");
    gemm(ga, DType::BF16, dt(out_dtype), false, false, s);
  });
}

int capgen_train_step_indexed(capgen_t* h, const void* feat_store, int feats_dtype, const float* pos_store,
                              int n_images, const int32_t* img_idx, const int32_t* caps, int B, int N, int T,
                              float* loss_out, void* stream) {
  return guarded([&] {
    set_device(h);
    require(n_images >= 1, "train_step_indexed: empty store");
    h->in_idx = img_idx;
    h->in_n_img = n_images;
    try {
      h->train_step(feat_store, dt(feats_dtype), pos_store, caps, B, N, T, loss_out, (hipStream_t)stream);
    } catch (...) {
      h->in_idx = nullptr;
      throw;
    }
    h->in_idx = nullptr;
    h->dp_check((hipStream_t)stream, loss_out);
  });
}

int capgen_rl_sample(capgen_t* h, const void* feats, int feats_dtype, const float* pos, const int32_t* caps, int B,
                     int N, int T, int64_t* sample_out, float* entropy_out, float* lm_loss_out, void* stream) {
  return guarded([&] {
    set_device(h);
    h->rl_sample(feats, dt(feats_dtype), pos, caps, B, N, T, sample_out, entropy_out, lm_loss_out, (hipStream_t)stream);
  });
}

int capgen_rl_finish(capgen_t* h, const float* scores, float structure_loss_weight, float* loss_out, int train,
                     void* stream) {
  return guarded([&] {
    set_device(h);
    h->rl_finish(scores, structure_loss_weight, loss_out, train != 0, (hipStream_t)stream);
  });
}

int capgen_scst_rewards(const int64_t* target, int64_t target_ld, const int64_t* sample, int64_t sample_ld, int B,
                        int L, int start_id, int end_id, int null_id, int64_t dot_id, double cider_w, double bleu_w,
                        double* out) {
  return guarded([&] {
    scst_rewards(target, target_ld, sample, sample_ld, B, L, start_id, end_id, null_id, dot_id, cider_w, bleu_w, out);
  });
}

int capgen_debug_attention(int dtype, int B, int H, int Lq, int Lk, int dk, const void* q, const void* k,
                           const void* v, const unsigned char* key_valid, int causal, float temperature, void* o,
                           float* probs, const void* dout, void* dq, void* dk_, void* dv, void* stream) {
  return guarded([&] {
    require(B >= 1 && H >= 1 && dk >= 1, "debug_attention: bad shape");
    const int64_t ld = (int64_t)H * dk;
    AttnGeom g;
    g.B = B, g.H = H, g.Lq = Lq, g.Lk = Lk, g.dk = dk;
    g.q = q, g.q_ld = ld, g.q_bs = Lq * ld;
    g.k = k, g.k_ld = ld, g.k_bs = Lk * ld;
    g.v = v, g.v_ld = ld, g.v_bs = Lk * ld;
    g.o_ld = ld, g.o_bs = Lq * ld;
    g.key_valid = key_valid, g.kv_bs = Lk;
    g.causal = causal;
    g.temperature = temperature;
    hipStream_t s = (hipStream_t)stream;
    attention_fwd(g, o, probs, dt(dtype), s);
    if (dout) attention_bwd(g, probs, dout, dq, dk_, dv, dt(dtype), s);
  });
}

// the test hooks' weights in the fronts' tiled layout (a per-process scratch, grown as needed)
static const bf16* debug_tiles(const bf16* W, int rows, hipStream_t s) {
  static bf16* buf = nullptr;
  static size_t cap = 0;
  const size_t need = (size_t)rows * 512 * 2;
  if (need > cap) {
    CAPGEN_HIP(hipDeviceSynchronize());  // (the previous scratch may still be read)
    if (buf) CAPGEN_HIP(hipFree(buf));
    CAPGEN_HIP(hipMalloc(&buf, need));
    cap = need;
  }
  qkv_tile_weights(W, rows, 512, buf, s);
  return buf;
}

int capgen_debug_qkv_attention(int B, int L, int H, const void* X, const void* W, void* qkv, void* o,
                               const unsigned char* key_valid, const int32_t* key_ids, int pad_idx, int causal,
                               void* stream) {
  return guarded([&] {
    require(B >= 1 && L >= 1 && H >= 1, "debug_qkv_attention: bad shape");
    const int d = H * 64;
    QkvAttn qa;
    AttnGeom& g = qa.g;
    g.B = B, g.H = H, g.Lq = L, g.Lk = L, g.dk = 64;
    g.q = qkv, g.q_ld = 3 * d, g.q_bs = (int64_t)L * 3 * d;
    g.k = (const bf16*)qkv + d, g.k_ld = 3 * d, g.k_bs = (int64_t)L * 3 * d;
    g.v = (const bf16*)qkv + 2 * d, g.v_ld = 3 * d, g.v_bs = (int64_t)L * 3 * d;
    g.o_ld = d, g.o_bs = (int64_t)L * d;
    g.key_valid = key_valid, g.kv_bs = L, g.key_ids = key_ids, g.kid_bs = L, g.pad_idx = pad_idx, g.causal = causal;
    g.temperature = 8.f;  // sqrt(64)
    qa.X = (const bf16*)X, qa.ldx = d, qa.W = debug_tiles((const bf16*)W, 3 * d, (hipStream_t)stream), qa.d = d;
    qa.qkv = (bf16*)qkv, qa.ldqkv = 3 * d, qa.o = (bf16*)o;
    qkv_attn_fwd(qa, (hipStream_t)stream);
  });
}

int capgen_debug_cross_attention(int B, int Lq, int Lk, int H, const void* X, const void* Wq, const void* KV, void* q,
                                 void* o, const unsigned char* key_valid, void* stream) {
  return guarded([&] {
    require(B >= 1 && Lq >= 1 && Lk >= 1 && H >= 1, "debug_cross_attention: bad shape");
    const int d = H * 64;
    QkvAttn qa;
    AttnGeom& g = qa.g;
    g.B = B, g.H = H, g.Lq = Lq, g.Lk = Lk, g.dk = 64;
    g.q = q, g.q_ld = d, g.q_bs = (int64_t)Lq * d;
    g.k = KV, g.k_ld = 2 * d, g.k_bs = (int64_t)Lk * 2 * d;
    g.v = (const bf16*)KV + d, g.v_ld = 2 * d, g.v_bs = (int64_t)Lk * 2 * d;
    g.o_ld = d, g.o_bs = (int64_t)Lq * d;
    g.key_valid = key_valid, g.kv_bs = Lk;
    g.temperature = 8.f;
    qa.cross = 1;
    qa.X = (const bf16*)X, qa.ldx = d, qa.W = debug_tiles((const bf16*)Wq, d, (hipStream_t)stream), qa.d = d;
    qa.qkv = (bf16*)q, qa.ldqkv = d, qa.o = (bf16*)o;
    qkv_attn_fwd(qa, (hipStream_t)stream);
  });
}

int capgen_debug_attention_bwd_wo(int B, int Lq, int Lk, int H, const void* q, const void* k, const void* v,
                                  const unsigned char* key_valid, int causal, const void* dA, const void* Wo, void* dq,
                                  void* dk, void* dv, void* stream) {
  return guarded([&] {
    require(B >= 1 && Lq >= 1 && Lk >= 1 && H * 64 == 512, "debug_attention_bwd_wo: bad shape (H * 64 = 512)");
    const int d = H * 64;
    const hipStream_t s = (hipStream_t)stream;
    static bf16* wt = nullptr;  // (the test hook's tiled Wo^T scratch)
    if (!wt) CAPGEN_HIP(hipMalloc(&wt, (size_t)512 * 512 * 2));
    qkv_tile_weights_t((const bf16*)Wo, 512, wt, s);
    QkvBwd qb;
    AttnGeom& g = qb.g;
    g.B = B, g.H = H, g.Lq = Lq, g.Lk = Lk, g.dk = 64;
    g.q = q, g.q_ld = d, g.q_bs = (int64_t)Lq * d;
    g.k = k, g.k_ld = d, g.k_bs = (int64_t)Lk * d;
    g.v = v, g.v_ld = d, g.v_bs = (int64_t)Lk * d;
    g.o_ld = d, g.o_bs = (int64_t)Lq * d;
    if (key_valid) g.key_valid = key_valid, g.kv_bs = Lk;
    g.causal = causal;
    g.temperature = 8.f;
    qb.dA = (const bf16*)dA, qb.ldda = d, qb.Wt = wt;
    qb.dq = (bf16*)dq, qb.dk = (bf16*)dk, qb.dv = (bf16*)dv;
    qkv_attn_bwd(qb, s);
  });
}

int capgen_debug_gemm_variant(int v) {
  return guarded([&] { gemm_set_variant(v); });
}

int capgen_debug_copy_buffer(capgen_t* h, int which, void* host_dst, int64_t bytes) {
  return guarded([&] {
    set_device(h);
    require(h->ws != nullptr, "debug_copy_buffer: no workspace yet");
    const int Le = h->L.Le;
    void* src = which == 0 ? h->a.tmp : which == 1 ? h->a.gOut : which == 2 ? h->a.gRes : which == 3 ? h->a.gKV
              : which == 4 ? h->a.genc[Le - 1].gH : which == 5 ? h->a.genc[Le - 1].gAf
              : which == 6 ? h->a.genc[Le - 1].gA1 : which == 7 ? h->a.genc[Le - 1].gQKV
              // 32 + 8 l + j: encoder block l's per-block gradient buffers (never overwritten later in
              // the backward): j = 0 gAf, 1 gH, 2 gA1, 3 gATT1, 4 gQKV
              : which >= 32 && (which - 32) / 8 < Le && (which - 32) % 8 < 5
                  ? (&h->a.genc[(which - 32) / 8].gAf)[(which - 32) % 8 == 0 ? 0 : (which - 32) % 8 == 1 ? 1
                                                        : (which - 32) % 8 == 2 ? 2 : (which - 32) % 8 == 3 ? 3 : 4]
              // 80 + l: the forward's encoder activations X[l] (l = 0 .. Le: embedding output .. encoder output)
              : which >= 80 && which - 80 <= Le ? h->a.X[which - 80]
              // 128 + 8 l + j: encoder block l's saved forward tensors: j = 0 att, 1 v1, 2 m1, 3 r1, 4 Y,
              // 5 v2, 6 m2, 7 r2
              : which >= 128 && (which - 128) / 8 < Le
                  ? ((which - 128) % 8 == 0 ? h->a.enc[(which - 128) / 8].att
                     : (which - 128) % 8 == 1 ? h->a.enc[(which - 128) / 8].v1
                     : (which - 128) % 8 == 2 ? (void*)h->a.enc[(which - 128) / 8].m1
                     : (which - 128) % 8 == 3 ? (void*)h->a.enc[(which - 128) / 8].r1
                     : (which - 128) % 8 == 4 ? h->a.enc[(which - 128) / 8].Y
                     : (which - 128) % 8 == 5 ? h->a.enc[(which - 128) / 8].v2
                     : (which - 128) % 8 == 6 ? (void*)h->a.enc[(which - 128) / 8].m2
                                             : (void*)h->a.enc[(which - 128) / 8].r2)
              // 200 + l / 216 + l: encoder / decoder block l's FFN hidden activations relu(x W1^T + b1)
              // (the ReLU mask the backward applies)
              : which >= 200 && which - 200 < Le ? h->a.enc[which - 200].H
              : which >= 216 && which - 216 < h->L.Ld ? h->a.dec[which - 216].H
                  : nullptr;
    require(src != nullptr,
            "debug_copy_buffer: which in 0..7, 32 + 8 l + 0..4, 80 + 0..Le, 128 + 8 l + 0..7, 200 + l, 216 + l");
    hz::host_sync(nullptr);
    CAPGEN_HIP(hipMemcpy(host_dst, src, (size_t)bytes, hipMemcpyDeviceToHost));
  });
}

int capgen_debug_gemm_timing_buf(void* dev_buf) {
  return guarded([&] { gemm_set_timing_buf(reinterpret_cast<uint64_t*>(dev_buf)); });
}

int capgen_debug_splitk_diag(int* out4, int reset) {
  return guarded([&] { gemm_splitk_diag(out4, reset != 0); });
}

int capgen_debug_splitk_protocol(int proto) {
  return guarded([&] {
    require(proto >= 0 && proto < 8192, "debug_splitk_protocol: bits 0..12 only (10-12: ablation build)");
    gemm_set_splitk_protocol(proto);
  });
}

int capgen_tune_load(const char* path) {
  int n = -1;
  const int rc = guarded([&] {
    require(path != nullptr, "tune_load: null path");
    n = gemm_tune_load(path);
  });
  return rc ? -2 : n;
}
int capgen_tune_save(const char* path) {
  int n = -1;
  const int rc = guarded([&] {
    require(path != nullptr, "tune_save: null path");
    n = gemm_tune_save(path);
    require(n >= 0, std::string("tune_save: cannot write ") + path);
  });
  return rc ? -2 : n;
}
int capgen_tune_live_count(void) { return gemm_tune_live_count(); }

int capgen_debug_hazard(int op, char* report, int cap, int* n_conflicts) {
  return guarded([&] {
    require(op >= 0 && op <= 2, "debug_hazard: op 0 (off), 1 (on + clear) or 2 (check)");
    if (op == 0) return hz::enable(false);
    if (op == 1) {
      hz::reset();
      return hz::enable(true);
    }
    std::string rep;
    const int n = hz::check(&rep);
    if (n_conflicts) *n_conflicts = n;
    if (report && cap > 0) {
      const size_t k = std::min<size_t>(rep.size(), (size_t)cap - 1);
      std::memcpy(report, rep.data(), k);
      report[k] = 0;
    }
  });
}
int capgen_debug_collectives(capgen_t* h, int op, char* out, int cap) {
  return guarded([&] {
    require(h != nullptr, "null engine handle");
    require(op >= 0 && op <= 2, "debug_collectives: op 0 (off), 1 (on + clear) or 2 (dump)");
    if (op < 2) {
      h->coll_log_on = op == 1;
      h->coll_log.clear();
      return;
    }
    std::string all;
    for (auto& l : h->coll_log) all += l + "\n";
    if (out && cap > 0) {
      const size_t k = std::min<size_t>(all.size(), (size_t)cap - 1);
      std::memcpy(out, all.data(), k);
      out[k] = 0;
    }
  });
}

int capgen_debug_stamps(capgen_t* h, int op, double* out, int cap, char* names, int names_cap) {
  int count = 0;
  const int rc = guarded([&] {
    require(h != nullptr, "null engine handle");
    require(op >= 0 && op <= 3, "debug_stamps: op 0 (off), 1 (on), 2 (read), 3 (arm)");
    set_device(h);
    if (op == 0 || op == 1) {
      hz::host_sync(nullptr);
      h->stamp_on = op == 1;
      if (h->stamp_on && !h->stamp_ring)
        CAPGEN_HIP(hipMalloc(&h->stamp_ring, (size_t)capgen_engine::kStampSlots * 16 * sizeof(uint64_t)));
      h->drop_graph();  // a captured forward holds its launches' stamp pointers
    }
    if (op == 3 || op == 1) {
      hz::host_sync(nullptr);
      if (h->stamp_ring) CAPGEN_HIP(hipMemset(h->stamp_ring, 0, (size_t)capgen_engine::kStampSlots * 16 * sizeof(uint64_t)));
      CAPGEN_HIP(hipDeviceSynchronize());
    }
    if (op == 2) {
      require(h->stamp_ring != nullptr, "debug_stamps: not enabled");
      hz::host_sync(nullptr);
      std::vector<uint64_t> ring((size_t)h->stamp_max * 16);
      CAPGEN_HIP(hipMemcpy(ring.data(), h->stamp_ring, ring.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
      std::string all;
      for (int i = 0; i < h->stamp_max && 2 * i + 1 < cap; ++i) {
        uint64_t e = 0;
        for (int k = 1; k <= 8; ++k) e = std::max(e, ring[(size_t)i * 16 + k]);
        out[2 * i] = (double)ring[(size_t)i * 16] * 0.01;  // 100 MHz ticks -> us
        out[2 * i + 1] = (double)e * 0.01;
        all += (i < (int)h->stamp_names.size() ? h->stamp_names[i] : std::string("?")) + "\n";
        ++count;
      }
      if (names && names_cap > 0) {
        const size_t k = std::min<size_t>(all.size(), (size_t)names_cap - 1);
        std::memcpy(names, all.data(), k);
        names[k] = 0;
      }
    }
  });
  return rc ? -1 : count;
}

int capgen_debug_side_delay(double us) {
  return guarded([&] { hz::set_delay_us(us); });
}

int capgen_dp_unique_id(char out[128]) {
  return guarded([&] {
    ncclUniqueId id;
    NCCL_CHECK(ncclGetUniqueId(&id));
    std::memcpy(out, id.internal, 128);
  });
}

int capgen_dp_init(capgen_t* h, const char id[128], int rank, int world) {
  return guarded([&] {
    set_device(h);
    require(world >= 1 && rank >= 0 && rank < world, "dp_init: bad rank/world");
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, 128);
    if (h->comm) ncclCommDestroy(h->comm);
    NCCL_CHECK(ncclCommInitRank(&h->comm, world, uid, rank));
    h->rank = rank, h->world = world;
    h->drop_graph();
    // replicate rank 0's parameters
    NCCL_CHECK(ncclBroadcast(h->params, h->params, (size_t)h->L.total, ncclFloat, 0, h->comm, h->es));
    h->refresh_shadow(h->es);
    hz::host_sync(h->es);
  });
}

int capgen_dp_comm_info(capgen_t* h, int* nranks, int* rank) {
  return guarded([&] {
    int n = 0, r = 0;
    if (h->comm) {
      NCCL_CHECK(ncclCommCount(h->comm, &n));
      NCCL_CHECK(ncclCommUserRank(h->comm, &r));
    }
    if (nranks) *nranks = n;
    if (rank) *rank = r;
  });
}

int capgen_dp_check(capgen_t* h, const float* loss, void* stream) {
  return guarded([&] {
    set_device(h);
    require(h->comm != nullptr, "dp_check: no communicator (capgen_dp_init first)");
    h->dp_check((hipStream_t)stream, loss, /*force=*/true);
  });
}

int capgen_params_checksum(capgen_t* h, uint64_t* out) {
  return guarded([&] {
    set_device(h);
    require(out != nullptr, "params_checksum: null output");
    hz::host_sync(h->es);
    hz::host_sync(h->ec);
    *out = arena_checksum(h->params, (size_t)h->L.total, h->es);
  });
}

int capgen_dp_sync_adam_state(capgen_t* h) {
  return guarded([&] {
    set_device(h);
    hz::host_sync(h->es);
    hz::host_sync(h->ec);
    const int zw = h->zworld();
    if (!h->comm || zw <= 1 || !h->zsharded()) return;
    for (auto& b : h->zbuckets) {
      if (b[1] % (4 * zw)) continue;  // updated by all-reduce + full Adam: already replicated
      const int64_t c = b[1] / zw, o = b[0] + (int64_t)h->zrank() * c;
      NCCL_CHECK(ncclAllGather(h->am + o, h->am + b[0], (size_t)c, ncclFloat, h->comm, h->es));
      NCCL_CHECK(ncclAllGather(h->av + o, h->av + b[0], (size_t)c, ncclFloat, h->comm, h->es));
    }
    h->moments_sharded = false;
    hz::host_sync(h->es);
  });
}

int capgen_dp_buckets(capgen_t* h, int64_t* offs, int64_t* counts, int cap, int* n) {
  return guarded([&] {
    require(h != nullptr && n != nullptr, "dp_buckets: null argument");
    require((int)h->zbuckets.size() <= cap, "dp_buckets: capacity too small");
    for (size_t i = 0; i < h->zbuckets.size(); ++i) offs[i] = h->zbuckets[i][0], counts[i] = h->zbuckets[i][1];
    *n = (int)h->zbuckets.size();
  });
}

int capgen_dp_debug_shard(capgen_t* h, int rank, int world) {
  return guarded([&] {
    require(h != nullptr, "null engine handle");
    require(world <= 1 || (rank >= 0 && rank < world), "dp_debug_shard: bad rank/world");
    require(world <= 1 || !h->comm, "dp_debug_shard: not with a communicator");
    h->zemu_rank = world > 1 ? rank : 0;
    h->zemu_world = world > 1 ? world : 1;
  });
}

int capgen_dp_set_global_count(capgen_t* h, float count) {
  return guarded([&] {
    set_device(h);
    // the previous step's asynchronous copy may still be queued: it must read the old value
    CAPGEN_HIP(hipEventSynchronize(h->ev_count));
    if (h->count_override != (count > 0.f)) h->drop_graph();  // the forward graph's count source changes
    h->count_override = count > 0.f;
    *h->count_host = count;
  });
}

}  // extern "C"
