// capgen — bf16 MFMA GEMM for gfx950, all three training layouts in one kernel template.
//
//   NT (forward  X.W^T)    : A [M][K], B [N][K]   both K-contiguous
//   NN (input grad dY.W)   : A [M][K], B [K][N]   B row-contiguous   (TB)
//   TN (weight grad dY^T.X): A [K][M], B [K][N]   both row-contiguous (TA, TB)
//
// Data movement.  Every operand tile is moved HBM/L2 -> LDS by global_load_lds_dwordx4
// (LDS-DMA, no staging registers) in its NATIVE layout, three stages deep: the DMA for
// K-tile kt+2 is in flight while tile kt is multiplied, retired by a counted
// `s_waitcnt vmcnt(loads per tile)` + raw s_barrier (never vmcnt(0) in the loop).
// LDS-DMA writes lane-linearly, so the bank-conflict swizzles are applied to the
// per-lane SOURCE address and undone on the fragment read (same involution).
// Out-of-range rows / K columns read a device zero page (no OOB access, exact K tails).
//
// Fragments.  K-contiguous images (128-B rows) are read with two ds_read_b64, XOR-
// swizzled in 16-B chunks by ((row>>1)&7).  Row-contiguous images are read with two
// ds_read_b64_tr_b16 (CDNA4 LDS transpose read), XOR-swizzled per K row.  Within each
// 32-deep v_mfma_f32_16x16x32_bf16 step, lane group g = lane>>4 carries k = 4g..4g+3
// (elements 0-3) and 16+4g..16+4g+3 (elements 4-7) for BOTH operands — the same K
// permutation on A and B leaves the dot product unchanged and makes every tr read of a
// half-wave cover 8 consecutive K rows (conflict free).  NT, NN and TN therefore run at
// the same LDS cost.
//
// Epilogue.  The MFMA is issued as B.A (operands swapped) so each lane ends with 4
// CONSECUTIVE output columns of one row: bias/relu-mask/accumulate/convert are applied
// on 4-wide vectors and stored as one 8-B (bf16) or 16-B (f32) write.
//
// Tiles BMxBNx64, 256 threads = 2x2 wave64s; blocks remapped so consecutive tiles (sharing
// an A row-panel) land on the same XCD L2.
#include <chrono>
#include <algorithm>
#include <dlfcn.h>
#include <string>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include <cstring>
#include "gemm.h"
#include "hazard.h"
#include "gemm_tile.h"
#include "tune_parse.h"

namespace capgen {

void gemm_hz_regions(const GemmArgs& g, DType in, DType out, bool ta, bool tb, std::vector<hz::Rgn>& v);  // gemm.hip

namespace {
void* g_zero_page[64] = {};
}  // namespace


template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int STAGES, int KG = 1>
__global__ void __launch_bounds__(64 * WM * WN * KG) gemm_bf16_kernel(GemmArgs g, int tiles_n, int nblk,
                                                                     const void* zero, int splitk, float* ws,
                                                                     int* tile_cnt, int group_m, int proto) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<TA, TB, BM, BN, WM, WN, STAGES, KG>::SMEM];
  StampScope stamp_scope(g.stamp);
  // critical-path launch (GemmArgs::prio): beside the side streams' weight-gradient / Adam waves
  // on the same CUs, the SIMD arbiter issues this kernel's instructions first
  if (g.prio) __builtin_amdgcn_s_setprio(3);
  const int slot = xcd_slot(blockIdx.x, nblk);
  const int tile = slot / splitk, split = slot % splitk;  // split-K slices of a tile are adjacent
  // tiles in column-major groups of group_m tile rows: an XCD's contiguous slot range covers a
  // compact 2D block of the output (fewer distinct A row panels + B column panels per L2)
  int mt = tile / tiles_n, nt = tile % tiles_n;
  if (group_m > 1) {
    const int tiles_m = (g.M + BM - 1) / BM, per = group_m * tiles_n, first = (tile / per) * group_m;
    const int gsz = min(tiles_m - first, group_m), r = tile % per;
    mt = first + r % gsz, nt = r / gsz;
  }
  gemm_tile<TO, TA, TB, BM, BN, WM, WN, STAGES, KG>(g, mt, nt, tile, split, splitk, zero, ws, tile_cnt, smem, proto);
}

// Grouped launch: up to kMaxGroup independent GEMMs of one layout (e.g. every weight gradient
// of a transformer block), each with its own M/N/pointers, tiles laid out problem after
// problem; one launch instead of one per weight, and a grid that fills the chip.
// G < nblk: a capped grid, each workgroup looping over the tiles b, b + G, ... (G % 8 == 0
// keeps every iteration on the workgroup's XCD).
template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int STAGES>
__global__ void __launch_bounds__(64 * WM * WN) gemm_bf16_grouped_kernel(GemmGroup gg, int nblk, int G,
                                                                        const void* zero) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<TA, TB, BM, BN, WM, WN, STAGES>::SMEM];
  StampScope stamp_scope(gg.p[0].stamp);
  for (int b = blockIdx.x; b < nblk; b += G) {
    if (b != (int)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
    const int slot = xcd_slot(b, nblk);
    int q = 0;
    while (q + 1 < gg.n && slot >= gg.start[q + 1]) ++q;
    const int tile = slot - gg.start[q];
    const int mt = tile / gg.tiles_n[q], nt = tile % gg.tiles_n[q];
    gemm_tile<TO, TA, TB, BM, BN, WM, WN, STAGES>(gg.p[q], mt, nt, tile, 0, 1, zero, nullptr, nullptr, smem);
  }
}

// The same, with the group description read from a device-resident table (grouped_args_dev): the
// launch carries one pointer instead of ~1.7 KB of kernel arguments (host enqueue cost)
template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int STAGES>
__global__ void __launch_bounds__(64 * WM * WN) gemm_bf16_grouped_dev_kernel(const GemmGroup* __restrict__ ggp,
                                                                            int nblk, int G, const void* zero) {
  __shared__ __attribute__((aligned(1024))) char smem[TileCfg<TA, TB, BM, BN, WM, WN, STAGES>::SMEM];
  const GemmGroup& gg = *ggp;
  StampScope stamp_scope(gg.p[0].stamp);
  for (int b = blockIdx.x; b < nblk; b += G) {
    if (b != (int)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
    const int slot = xcd_slot(b, nblk);
    int q = 0;
    while (q + 1 < gg.n && slot >= gg.start[q + 1]) ++q;
    const int tile = slot - gg.start[q];
    const int mt = tile / gg.tiles_n[q], nt = tile % gg.tiles_n[q];
    gemm_tile<TO, TA, TB, BM, BN, WM, WN, STAGES>(gg.p[q], mt, nt, tile, 0, 1, zero, nullptr, nullptr, smem);
  }
}

// split-K f32 workspaces, one per stream (GEMMs on different streams may run concurrently)
struct Workspace {
  float* p = nullptr;
  size_t bytes = 0;
  int* cnt = nullptr;  // per-tile arrival counters (zero between launches)
};
constexpr int kMaxTiles = 1 << 16;
std::map<hipStream_t, Workspace> g_ws;
// split-K hand-off protocol (diagnostic; 0 = production, see gemm_tile): bit 0 writer release,
// bit 1 no reader acquire, bit 2 sc1 slab loads, bit 3 per-launch ticket memset, bit 4 ticket
// re-armed by a relaxed atomic store (round 1: 2|4|16)
int g_splitk_proto = 0;  // (debug build: Knob::SplitkProto, read at gemm_init)
std::mutex g_ws_mu;
uint64_t* g_timing_buf = nullptr;  // ablation build, protocol bit 4096 (gemm_set_timing_buf)

// make sure the stream's split-K workspace holds `bytes` (never called inside a capture)
void ensure_ws(hipStream_t s, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Workspace& w = g_ws[s];
  if (!w.cnt) {
    CAPGEN_HIP(hipMalloc(&w.cnt, kMaxTiles * sizeof(int)));
    // on the stream itself: a null-stream hipMemset is not ordered before work on the
    // (non-blocking) engine streams, and a split-K launch reading stale tickets combines the
    // wrong slices (seen as a rare train_step vs forward/backward mismatch)
    CAPGEN_HIP(hipMemsetAsync(w.cnt, 0, kMaxTiles * sizeof(int), s));
  }
  if (w.bytes >= bytes) return;
  // a grown workspace retires the old one without freeing it: a graph captured earlier on
  // this stream (the replayed forward) still holds its address
  static std::vector<float*> retired;
  if (w.p) retired.push_back(w.p);
  CAPGEN_HIP(hipMalloc(&w.p, bytes));
  w.bytes = bytes;
}
Workspace get_ws(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  auto it = g_ws.find(s);
  return it == g_ws.end() ? Workspace{} : it->second;
}

template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int ST, int KG = 1>
static void launch_cfg(const GemmArgs& g, hipStream_t s, int splitk) {
  require(KG == 1 || splitk == 1, "gemm: k-group variants run without grid split-K");
  const int tn = (g.N + BN - 1) / BN, tm = (g.M + BM - 1) / BM;
  const int nblk = tn * tm * splitk;
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  float* ws = nullptr;
  int* cnt = nullptr;
  if (splitk > 1) {
    const size_t bytes = (size_t)tn * tm * splitk * BM * BN * sizeof(float);
    const Workspace w = get_ws(s);
    require(w.bytes >= bytes && w.cnt, "gemm: split-K workspace too small (tune outside capture)");
    require(tn * tm <= kMaxTiles, "gemm: too many tiles for split-K");
    ws = w.p, cnt = w.cnt;
    if (g_splitk_proto & 32) {  // diagnostic: rotate over 4 ticket arrays (kMaxTiles / 4 each)
      static std::map<hipStream_t, int> rot;
      cnt += (rot[s]++ & 3) * (kMaxTiles / 4);
      require(tn * tm <= kMaxTiles / 4, "gemm: too many tiles for ticket rotation");
    }
    // tickets: zeroed once at allocation and re-armed by each tile's last arriver (an atomic
    // exchange, gemm_tile); a per-launch memset (the guide's 'Re-initialise every call') costs
    // 6-40 us per launch as a separate node on ROCm 7 (tools/splitk_stress.py time) -- diagnostic
    // bit 8 of capgen_debug_splitk_protocol restores it
    if (g_splitk_proto & 8) CAPGEN_HIP(hipMemsetAsync(cnt, 0, (size_t)(tn * tm + 3) / 4 * 16, s));
  }
  // group_m ~ sqrt(tiles per XCD), so each XCD's tile block is about square
  int group_m = 0;
  {
    const double per_xcd = (double)tn * tm / 8.0;
    group_m = std::max(1, std::min(tm, (int)std::lround(std::sqrt(per_xcd))));
  }
  GemmArgs gk = g;
  if ((g_splitk_proto & 4096) && g_timing_buf) gk.stamp = g_timing_buf;  // (ablation build: phase timing)
  gemm_bf16_kernel<TO, TA, TB, BM, BN, WM, WN, ST, KG>
      <<<nblk, 64 * WM * WN * KG, 0, s>>>(gk, tn, nblk, g_zero_page[dev], splitk, ws, cnt, group_m, g_splitk_proto & ~8);
}

// split-K workspace bound for any variant (tiles up to 256x128)
size_t splitk_bytes(const GemmArgs& g, int splitk) {
  return (size_t)((g.M + 255) / 256 * 256) * ((g.N + 127) / 128 * 128) * splitk * sizeof(float);
}

int g_variant = 0;  // experiment selector (capgen_debug_gemm_variant); 0 = tuned/heuristic

// Tile / wave-grid / pipeline-depth variants.  Every variant accumulates the same K tiles
// in the same order with the same MFMA sequence, so results are bit-identical across
// variants: the choice is a pure speed decision (made per shape by the autotuner).
constexpr int NVARIANTS = 30;
const char* kVariantName[NVARIANTS + 1] = {"auto",        "128x128w4s3", "128x128w8s2",  "128x128w4s2",
                                           "128x64w4s2",  "64x128w4s2",  "64x64w4s2",    "64x64w4s3",
                                           "128x64w8s2",  "256x128w16s2", "128x128w16s2", "256x64w8s2",
                                           "64x64w4s4",   "64x64w4s6",   "128x64w4s4",   "64x128w4s4",
                                           "128x128w4s4", "32x64w4s2",   "64x32w4s2",    "32x32w4s2",
                                           "64x64w8s2",   "32x64w4s3",   "64x32w4s3",
                                           // k-group variants (TileCfg KG): 'k2' = 2 k-groups of the waves named
                                           "64x64w4k2s2", "64x64w4k2s3", "32x64w4k2s3", "64x64w4k4s2",
                                           "32x64w4k4s2", "128x64w4k2s2", "64x128w4k2s2", "32x64w4k2s2"};

// output tile width (columns) of each variant
constexpr int kVariantBN[NVARIANTS + 1] = {0,  128, 128, 128, 64, 128, 64, 64, 64, 128, 128, 64,
                                           64, 64,  64,  128, 128, 64, 32, 32, 64, 64,  32,
                                           64, 64,  64,  64,  64,  64, 128, 64};
// k-groups of each variant (grid split-K only for KG == 1)
constexpr int kVariantKG[NVARIANTS + 1] = {0, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                           1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 4, 4, 2, 2, 2};

// A tile whose output row segment is narrower than a 128-B cache line shares lines of C with
// its neighbour tile, which another workgroup -- possibly on another XCD -- writes in the same
// launch.  With a read-modify-write epilogue (beta: C is read first) each XCD's L2 then holds
// the whole line with the neighbour's half stale, and a later kernel on that XCD can read the
// stale half (measured: ~1 in 5 bf16 c2s backward passes differed run to run in the encoder
// gradients, tools/bwd_bisect.py).  Such variants are never chosen, so every line of C is
// written by exactly one workgroup.  CAPGEN_ALLOW_PARTIAL_LINES=1 lifts the rule (diagnostic).
template <typename TO>
static bool whole_lines(int v) {
  return knob(Knob::AllowPartialLines) || kVariantBN[v] * (int)sizeof(TO) >= 128;
}

template <typename TO, bool TA, bool TB>
static void launch_variant(int v, const GemmArgs& g, hipStream_t s, int sk = 1) {
  switch (v) {
    case 1: return launch_cfg<TO, TA, TB, 128, 128, 2, 2, 3>(g, s, sk);
    case 2: return launch_cfg<TO, TA, TB, 128, 128, 2, 4, 2>(g, s, sk);
    case 3: return launch_cfg<TO, TA, TB, 128, 128, 2, 2, 2>(g, s, sk);
    case 4: return launch_cfg<TO, TA, TB, 128, 64, 2, 2, 2>(g, s, sk);
    case 5: return launch_cfg<TO, TA, TB, 64, 128, 2, 2, 2>(g, s, sk);
    case 6: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 2>(g, s, sk);
    case 7: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 3>(g, s, sk);
    case 8: return launch_cfg<TO, TA, TB, 128, 64, 4, 2, 2>(g, s, sk);
    case 9: return launch_cfg<TO, TA, TB, 256, 128, 4, 4, 2>(g, s, sk);
    case 10: return launch_cfg<TO, TA, TB, 128, 128, 4, 4, 2>(g, s, sk);
    case 11: return launch_cfg<TO, TA, TB, 256, 64, 4, 2, 2>(g, s, sk);
    case 12: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 4>(g, s, sk);
    case 13: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 6>(g, s, sk);
    case 14: return launch_cfg<TO, TA, TB, 128, 64, 2, 2, 4>(g, s, sk);
    case 15: return launch_cfg<TO, TA, TB, 64, 128, 2, 2, 4>(g, s, sk);
    case 16: return launch_cfg<TO, TA, TB, 128, 128, 2, 2, 4>(g, s, sk);
    // small tiles: more workgroups per CU for the latency-bound small GEMMs of the step
    case 17: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 2>(g, s, sk);
    case 18: return launch_cfg<TO, TA, TB, 64, 32, 2, 2, 2>(g, s, sk);
    case 19: return launch_cfg<TO, TA, TB, 32, 32, 2, 2, 2>(g, s, sk);
    case 20: return launch_cfg<TO, TA, TB, 64, 64, 4, 2, 2>(g, s, sk);
    case 21: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 3>(g, s, sk);
    case 22: return launch_cfg<TO, TA, TB, 64, 32, 2, 2, 3>(g, s, sk);
    case 23: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 2, 2>(g, s, sk);
    case 24: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 3, 2>(g, s, sk);
    case 25: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 3, 2>(g, s, sk);
    case 26: return launch_cfg<TO, TA, TB, 64, 64, 2, 2, 2, 4>(g, s, sk);
    case 27: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 2, 4>(g, s, sk);
    case 28: return launch_cfg<TO, TA, TB, 128, 64, 2, 2, 2, 2>(g, s, sk);
    case 29: return launch_cfg<TO, TA, TB, 64, 128, 2, 2, 2, 2>(g, s, sk);
    case 30: return launch_cfg<TO, TA, TB, 32, 64, 2, 2, 2, 2>(g, s, sk);
    default: throw Error("gemm: unknown variant");
  }
}

int heuristic_variant(const GemmArgs& g) {
  const long b64 = (long)((g.M + 63) / 64) * ((g.N + 63) / 64);
  return b64 <= 4096 ? 6 : 3;
}

struct TuneKey {
  int M, N, K, ta, tb, out;
  bool operator<(const TuneKey& o) const {
    return std::tie(M, N, K, ta, tb, out) < std::tie(o.M, o.N, o.K, o.ta, o.tb, o.out);
  }
};
struct Choice {
  int variant, splitk;
};
std::map<TuneKey, Choice> g_tuned;
std::mutex g_tune_mu;
int g_live_tuned = 0;  // shapes (plain + grouped) tuned live in this process

bool autotune_enabled() {
  return knob(Knob::Autotune) != 0;
}

// Tuning-time clock of one (variant, split-K) candidate: 3 launches.  In the step every GEMM
// reads operands that are not in this XCD's L2 (the A operand was just written by the previous
// kernel -- possibly on another XCD -- and the weights were last touched a step ago), so the
// latency-bound small shapes run ~2x their L2-warm repeat time there (dec W2 1216x512x2048:
// 24.6 us in the step, 11.9 us repeated).  So each timed launch follows a 64 MB scrub write that
// evicts the L2s, and the tuner ranks candidates under the step's cache state (the warm repeat
// clock measured 3.236 vs 2.977 ms/step); the scrub itself is outside the timed span.
template <typename F>
static float tune_time(F&& launch, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  launch();  // warm-up (code, TLB)
  static std::map<int, void*> scrub;  // per device, never freed (tuning-time helper)
  constexpr size_t kScrub = 64u << 20;
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  void*& buf = scrub[dev];
  if (!buf) CAPGEN_HIP(hipMalloc(&buf, kScrub));
  float tot = 0.f;
  for (int r = 0; r < 3; ++r) {
    CAPGEN_HIP(hipMemsetAsync(buf, r, kScrub, s));
    CAPGEN_HIP(hipEventRecord(e0, s));
    launch();
    CAPGEN_HIP(hipEventRecord(e1, s));
    CAPGEN_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    CAPGEN_HIP(hipEventElapsedTime(&ms, e0, e1));
    tot += ms;
  }
  return tot;
}

template <typename TO, bool TA, bool TB>
static Choice tune(const GemmArgs& g, hipStream_t s) {
  // time every (variant, split-K) on a scratch output (inputs untouched, beta forced to 0)
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  GemmArgs t = g;
  void* scratch = nullptr;
  if (t.C2) t.C2 = nullptr, t.nsplit = 0, t.ldc = std::max<int64_t>(t.ldc, t.N);  // all columns to scratch
  CAPGEN_HIP(hipMalloc(&scratch, (size_t)t.M * t.ldc * sizeof(TO)));
  t.C = scratch;
  t.beta = 0;
  t.colsum = nullptr;
  t.stamp = nullptr;
  hipEvent_t e0, e1;
  CAPGEN_HIP(hipEventCreate(&e0));
  CAPGEN_HIP(hipEventCreate(&e1));
  Choice best{heuristic_variant(g), 1};
  float best_ms = 1e30f;
  const int nk = (g.K + BK - 1) / BK;
  // split-K factor cap 8.  Round 1 capped it at 2 because the bf16
  // step was not reproducible run to run with higher factors; the causes were a sub-line output
  // tile under a read-modify-write epilogue (whole_lines) and the combine's ticket re-arm /
  // missing acquire (gemm_tile) -- tools/step_det_probe.py: 0 of 60 diverging runs at cap 8 now.
  constexpr int max_sk = 8;
  for (int sk : {1, 2, 3, 4, 6, 8}) {
    if (sk > max_sk || (sk > 1 && nk < 4 * sk)) break;
    if (sk > 1) ensure_ws(s, splitk_bytes(g, sk));
    for (int v = 1; v <= NVARIANTS; ++v) {
      if (!whole_lines<TO>(v) || (sk > 1 && kVariantKG[v] > 1)) continue;
      const float ms = tune_time([&] { launch_variant<TO, TA, TB>(v, t, s, sk); }, s, e0, e1);
      if (ms < best_ms) best_ms = ms, best = Choice{v, sk};
    }
  }
  CAPGEN_HIP(hipEventDestroy(e0));
  CAPGEN_HIP(hipEventDestroy(e1));
  CAPGEN_HIP(hipFree(scratch));
  if (knob(Knob::AutotuneLog))
    std::fprintf(stderr, "[capgen gemm] M=%d N=%d K=%d ta=%d tb=%d out=%s -> %s splitk=%d (%.2f us)\n", g.M, g.N, g.K,
                 TA, TB, sizeof(TO) == 4 ? "f32" : "bf16", kVariantName[best.variant], best.splitk,
                 best_ms * 1e3f / 3);
  return best;
}

template <typename TO, bool TA, bool TB>
static void launch_bf16_tiles(const GemmArgs& g, hipStream_t s) {
  Choice c{g_variant % 100, std::max(1, g_variant / 100)};  // forced: variant + 100 * splitk
  if (TA && c.variant == 0) {  // debug build: weight-gradient (TN) GEMMs on a fixed variant
    const int dwv = knob(Knob::DwVariant);
    if (dwv) c = Choice{dwv % 100, std::max(1, dwv / 100)};
  }
  // debug build: CAPGEN_GEMM_FORCE="M,N,K,ta,tb,v[;...]" pins one shape's choice (variant v +
  // 100 * split-K), e.g. to A/B a critical-path GEMM in the step rather than alone
  static const std::map<TuneKey, int> forced = [] {
    std::map<TuneKey, int> m;
    if (const char* e = debug_build() ? std::getenv("CAPGEN_GEMM_FORCE") : nullptr) {
      int M, N, K, ta, tb, v, n = 0;
      for (const char* p = e; *p;) {
        if (std::sscanf(p, "%d,%d,%d,%d,%d,%d%n", &M, &N, &K, &ta, &tb, &v, &n) != 6) break;
        m[TuneKey{M, N, K, ta, tb, 2}] = v, m[TuneKey{M, N, K, ta, tb, 4}] = v;
        p += n;
        if (*p == ';') ++p;
      }
    }
    return m;
  }();
  if (c.variant == 0 && !forced.empty()) {
    auto it = forced.find(TuneKey{g.M, g.N, g.K, TA, TB, (int)sizeof(TO)});
    if (it != forced.end()) c = Choice{it->second % 100, std::max(1, it->second / 100)};
  }
  if (c.splitk > 1) ensure_ws(s, splitk_bytes(g, c.splitk));
  if (c.variant == 0) {
    c.variant = heuristic_variant(g);
    TuneKey key{g.M, g.N, g.K, TA, TB, (int)sizeof(TO)};
    std::lock_guard<std::mutex> lk(g_tune_mu);
    auto it = g_tuned.find(key);  // tuned in this process or loaded from the persisted table
    if (it != g_tuned.end()) {
      c = it->second;
    } else if (autotune_enabled()) {
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      CAPGEN_HIP(hipStreamIsCapturing(s, &st));
      if (st == hipStreamCaptureStatusNone) {
        // a shape the table does not hold: tune it on an idle device (every stream drained, so
        // no concurrent kernel shares the CUs or the caches with the candidates' clock, and the
        // candidates run strictly between the work issued before and after this call)
        CAPGEN_HIP(hipDeviceSynchronize());
        c = g_tuned[key] = tune<TO, TA, TB>(g, s);
        CAPGEN_HIP(hipStreamSynchronize(s));
        ++g_live_tuned;
      }
    }
  }
  if (c.splitk > 1) {
    const size_t bytes = splitk_bytes(g, c.splitk);
    const Workspace w = get_ws(s);
    if (!(w.cnt && w.bytes >= bytes)) {  // (the common case skips the capture query: host time)
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      CAPGEN_HIP(hipStreamIsCapturing(s, &st));
      if (st == hipStreamCaptureStatusNone) ensure_ws(s, bytes);
      else c.splitk = 1;  // no allocation inside a capture
    }
  }
  launch_variant<TO, TA, TB>(c.variant, g, s, c.splitk);
}

template <typename TO>
static void launch_bf16_layout(const GemmArgs& g, bool ta, bool tb, hipStream_t s) {
  if (!ta && !tb) launch_bf16_tiles<TO, false, false>(g, s);
  else if (!ta && tb) launch_bf16_tiles<TO, false, true>(g, s);
  else if (ta && !tb) launch_bf16_tiles<TO, true, false>(g, s);
  else launch_bf16_tiles<TO, true, true>(g, s);
}

// ---- grouped launch ---------------------------------------------------------------------
// Device-resident copies of grouped-launch descriptions, keyed by their bytes: a step issues the
// same ~16 groups every time (same pointers), so each is copied to the device once and later
// launches pass its address.  Entries are never freed (a captured graph may hold one); the table
// is bounded (kGroupTableCap entries per device, then launches fall back to by-value arguments).
// CAPGEN_GROUP_ARGS_DEV=0 restores by-value arguments.
constexpr int kGroupTableCap = 2048;
struct GroupTable {
  std::map<uint64_t, std::vector<std::pair<GemmGroup, const GemmGroup*>>> by_hash;
  GemmGroup* dev = nullptr;
  int used = 0;
};
GroupTable g_group_table[64];
std::mutex g_group_table_mu;

const GemmGroup* grouped_args_dev(const GemmGroup& gg, int dev, hipStream_t s) {
  const unsigned char* b = reinterpret_cast<const unsigned char*>(&gg);
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < sizeof(GemmGroup); ++i) h = (h ^ b[i]) * 1099511628211ull;
  std::lock_guard<std::mutex> lk(g_group_table_mu);
  GroupTable& t = g_group_table[dev];
  auto& bucket = t.by_hash[h];
  for (auto& e : bucket)
    if (std::memcmp(&e.first, &gg, sizeof(GemmGroup)) == 0) return e.second;
  if (t.used >= kGroupTableCap) return nullptr;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  CAPGEN_HIP(hipStreamIsCapturing(s, &st));
  if (st != hipStreamCaptureStatusNone) return nullptr;  // no synchronous copy inside a capture
  if (!t.dev) CAPGEN_HIP(hipMalloc(&t.dev, sizeof(GemmGroup) * kGroupTableCap));
  GemmGroup* slot = t.dev + t.used++;
  // synchronous: complete before any later launch reads it; the slot is fresh (no reader yet)
  CAPGEN_HIP(hipMemcpy(slot, &gg, sizeof(GemmGroup), hipMemcpyHostToDevice));
  bucket.push_back({gg, slot});
  return slot;
}

template <typename TO, bool TA, bool TB, int BM, int BN, int WM, int WN, int ST>
static void launch_group_cfg(const GemmArgs* ps, int n, hipStream_t s) {
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  GemmGroup gg;  // (no padding bytes: gemm.h; unused problem slots stay value-initialised)
  gg.n = n;
  int tot = 0;
  for (int i = 0; i < n; ++i) {
    const int tn = (ps[i].N + BN - 1) / BN, tm = (ps[i].M + BM - 1) / BM;
    gg.start[i] = tot, gg.tiles_n[i] = tn, gg.p[i] = ps[i];
    tot += tn * tm;
  }
  gg.start[n] = tot;
  // the grouped (weight-gradient) grid is capped at one workgroup per CU, each looping over its
  // tiles: the side-stream dW work then leaves room on every CU for the critical stream's
  // latency-bound kernels (step 3.44-3.47 vs 3.54 ms uncapped; 64 workgroups: 3.75 ms, the dW
  // work becomes critical; round 4 re-sweep: 256 vs 192 / 320 / 128, tools/r04_dwgrid.sh).
  static const int cap = [] {
    int n = 0, dev = 0;
    CAPGEN_HIP(hipGetDevice(&dev));
    CAPGEN_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    return std::max(8, n / 8 * 8);
  }();
  const int G = cap > 0 ? std::min(tot, cap) : tot;
  if (const GemmGroup* d = grouped_args_dev(gg, dev, s))
    gemm_bf16_grouped_dev_kernel<TO, TA, TB, BM, BN, WM, WN, ST><<<G, 64 * WM * WN, 0, s>>>(d, tot, G, g_zero_page[dev]);
  else
    gemm_bf16_grouped_kernel<TO, TA, TB, BM, BN, WM, WN, ST><<<G, 64 * WM * WN, 0, s>>>(gg, tot, G, g_zero_page[dev]);
}

// the variants worth a grouped launch (many tiles already: no split-K)
constexpr int kGroupVariants[] = {6, 20, 17, 18, 19, 4, 8, 1, 3, 10};

template <typename TO, bool TA, bool TB>
static void launch_group_variant(int v, const GemmArgs* ps, int n, hipStream_t s) {
  switch (v) {
    case 1: return launch_group_cfg<TO, TA, TB, 128, 128, 2, 2, 3>(ps, n, s);
    case 3: return launch_group_cfg<TO, TA, TB, 128, 128, 2, 2, 2>(ps, n, s);
    case 4: return launch_group_cfg<TO, TA, TB, 128, 64, 2, 2, 2>(ps, n, s);
    case 6: return launch_group_cfg<TO, TA, TB, 64, 64, 2, 2, 2>(ps, n, s);
    case 8: return launch_group_cfg<TO, TA, TB, 128, 64, 4, 2, 2>(ps, n, s);
    case 10: return launch_group_cfg<TO, TA, TB, 128, 128, 4, 4, 2>(ps, n, s);
    case 17: return launch_group_cfg<TO, TA, TB, 32, 64, 2, 2, 2>(ps, n, s);
    case 18: return launch_group_cfg<TO, TA, TB, 64, 32, 2, 2, 2>(ps, n, s);
    case 19: return launch_group_cfg<TO, TA, TB, 32, 32, 2, 2, 2>(ps, n, s);
    case 20: return launch_group_cfg<TO, TA, TB, 64, 64, 4, 2, 2>(ps, n, s);
    default: throw Error("gemm_grouped: unknown variant");
  }
}

std::map<std::vector<int>, int> g_group_tuned;

template <typename TO, bool TA, bool TB>
static void launch_group(const GemmArgs* ps, int n, hipStream_t s) {
  std::vector<int> key{TA, TB, (int)sizeof(TO)};
  for (int i = 0; i < n; ++i) key.insert(key.end(), {ps[i].M, ps[i].N, ps[i].K});
  int v = g_variant % 100;
  if (v == 0) {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    auto it = g_group_tuned.find(key);
    if (it != g_group_tuned.end()) {
      v = it->second;
    } else {
      v = kGroupVariants[0];
      hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
      CAPGEN_HIP(hipStreamIsCapturing(s, &st));
      if (st == hipStreamCaptureStatusNone && autotune_enabled()) {
        CAPGEN_HIP(hipDeviceSynchronize());  // idle device (see launch_bf16_tiles)
        ++g_live_tuned;
        // time each variant on scratch outputs (inputs untouched, beta forced to 0)
        std::vector<GemmArgs> t(ps, ps + n);
        std::vector<void*> scratch(n);
        for (int i = 0; i < n; ++i) {
          CAPGEN_HIP(hipMalloc(&scratch[i], (size_t)t[i].M * t[i].ldc * sizeof(TO)));
          t[i].C = scratch[i], t[i].beta = 0, t[i].colsum = nullptr, t[i].stamp = nullptr;
        }
        hipEvent_t e0, e1;
        CAPGEN_HIP(hipEventCreate(&e0));
        CAPGEN_HIP(hipEventCreate(&e1));
        float best = 1e30f;
        for (int cand : kGroupVariants) {
          if (!whole_lines<TO>(cand)) continue;
          const float ms = tune_time([&] { launch_group_variant<TO, TA, TB>(cand, t.data(), n, s); }, s, e0, e1);
          if (ms < best) best = ms, v = cand;
        }
        CAPGEN_HIP(hipEventDestroy(e0));
        CAPGEN_HIP(hipEventDestroy(e1));
        for (void* p : scratch) CAPGEN_HIP(hipFree(p));
        CAPGEN_HIP(hipStreamSynchronize(s));
        g_group_tuned[key] = v;
        if (knob(Knob::AutotuneLog))
          std::fprintf(stderr, "[capgen gemm] group of %d (M=%d N=%d K=%d first) -> %s (%.2f us)\n", n, ps[0].M,
                       ps[0].N, ps[0].K, kVariantName[v], best * 1e3f / 3);
      }
    }
  }
  launch_group_variant<TO, TA, TB>(v, ps, n, s);
}

static void gemm_grouped_impl(const GemmArgs* ps, int n, DType out, bool ta, bool tb, hipStream_t s);
// debug build, Knob::HostTiming: average host time of a grouped launch, printed every 500 calls
void gemm_grouped(const GemmArgs* ps, int n, DType out, bool ta, bool tb, hipStream_t s) {
  if (!knob(Knob::HostTiming)) return gemm_grouped_impl(ps, n, out, ta, tb, s);
  static double tot = 0;
  static long cnt = 0;
  const auto t0 = std::chrono::steady_clock::now();
  gemm_grouped_impl(ps, n, out, ta, tb, s);
  tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  if (++cnt % 500 == 0) {
    std::fprintf(stderr, "[capgen host] gemm_grouped() call: %.2f us average over 500\n", tot / 500);
    tot = 0;
  }
}
static void gemm_grouped_impl(const GemmArgs* ps, int n, DType out, bool ta, bool tb, hipStream_t s) {
  require(n >= 1 && n <= kMaxGroup, "gemm_grouped: 1..kMaxGroup problems");
  if ((skip_mask() & 16) && out == DType::F32) return;  // (debug build: marginal-cost probes)
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  require(g_zero_page[dev] != nullptr, "gemm: gemm_init() not called on this device");
  std::vector<GemmArgs> pw(ps, ps + n);  // write-through default, as gemm_bf16
  for (auto& g : pw) {
    if (g.wt < 0) g.wt = wt_default();
    if ((int64_t)g.M * g.ldc * (int64_t)dsize(out) >= (int64_t)0x7FFFFFFF) g.wt = 0;
  }
  ps = pw.data();
  for (int i = 0; i < n; ++i) {
    const GemmArgs& g = ps[i];
    require(g.M > 0 && g.N > 0 && g.K > 0 && g.N % 4 == 0 && g.ldc % 4 == 0 && (g.aux == nullptr || g.ldaux % 4 == 0),
            "gemm_grouped: bad problem shape");
    require(((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0, "gemm_grouped: operands must be 16-B aligned");
  }
  if (hz::active()) {
    std::vector<hz::Rgn> v;
    for (int i = 0; i < n; ++i) gemm_hz_regions(ps[i], DType::BF16, out, ta, tb, v);
    hz::op(s, "gemm grouped (dW)", v.data(), v.size());
  }
  if (out == DType::F32) {
    if (ta && tb) launch_group<float, true, true>(ps, n, s);
    else if (!ta && tb) launch_group<float, false, true>(ps, n, s);
    else throw Error("gemm_grouped: layout not instantiated");
  } else {
    if (!ta && tb) launch_group<bf16, false, true>(ps, n, s);
    else if (!ta && !tb) launch_group<bf16, false, false>(ps, n, s);
    else throw Error("gemm_grouped: layout not instantiated");
  }
  CAPGEN_HIP(hipGetLastError());
}

// ---- persisted autotune table --------------------------------------------------------------
// Text, one choice per line:  g M N K ta tb out_bytes variant splitk
//                             G ta tb out_bytes n M1 N1 K1 ... Mn Nn Kn variant
int gemm_tune_load(const char* path) {
  FILE* f = std::fopen(path, "r");
  if (!f) return -1;
  std::lock_guard<std::mutex> lk(g_tune_mu);
  int n = 0;
  char line[1024];
  while (std::fgets(line, sizeof line, f)) {
    if (line[0] == 'g') {
      TuneLineG t;
      if (parse_tune_g(line + 1, NVARIANTS, &t)) {
        g_tuned.emplace(TuneKey{t.M, t.N, t.K, t.ta, t.tb, t.out}, Choice{t.variant, t.splitk});
        ++n;
      }
    } else if (line[0] == 'G') {
      std::vector<int> key;
      int var = 0;
      if (parse_tune_G(line + 1, kGroupVariants, (int)(sizeof kGroupVariants / sizeof kGroupVariants[0]), kMaxGroup,
                       &key, &var)) {
        g_group_tuned.emplace(key, var);
        ++n;
      }
    }
  }
  std::fclose(f);
  return n;
}

int gemm_tune_save(const char* path) {
  FILE* f = std::fopen(path, "w");
  if (!f) return -1;
  std::lock_guard<std::mutex> lk(g_tune_mu);
  std::fprintf(f, "# capgen bf16 GEMM autotune table (gfx950): g M N K ta tb out_bytes variant splitk | "
                  "G ta tb out_bytes n (M N K)xn variant\n");
  int n = 0;
  for (auto& kv : g_tuned) {
    const TuneKey& k = kv.first;
    std::fprintf(f, "g %d %d %d %d %d %d %d %d  # %s\n", k.M, k.N, k.K, k.ta, k.tb, k.out, kv.second.variant,
                 kv.second.splitk,
                 kv.second.variant >= 0 && kv.second.variant <= NVARIANTS ? kVariantName[kv.second.variant] : "?");
    ++n;
  }
  for (auto& kv : g_group_tuned) {
    const std::vector<int>& k = kv.first;
    std::fprintf(f, "G %d %d %d %d", k[0], k[1], k[2], (int)(k.size() - 3) / 3);
    for (size_t i = 3; i < k.size(); ++i) std::fprintf(f, " %d", k[i]);
    std::fprintf(f, " %d  # %s\n", kv.second,
                 kv.second >= 0 && kv.second <= NVARIANTS ? kVariantName[kv.second] : "?");
    ++n;
  }
  std::fclose(f);
  return n;
}

int gemm_tune_live_count() { return g_live_tuned; }

void gemm_set_variant(int v) { g_variant = v; }
void gemm_set_splitk_protocol(int p) {
  require(p == 0 || debug_build(), "split-K protocol bits are a debug-build diagnostic (libcapgen_debug.so)");
  g_splitk_proto = p;
}
void gemm_set_timing_buf(uint64_t* p) { g_timing_buf = p; }
void gemm_splitk_diag(int* out4, bool reset) {
  CAPGEN_HIP(hipDeviceSynchronize());
  CAPGEN_HIP(hipMemcpyFromSymbol(out4, HIP_SYMBOL(g_sk_diag), 4 * sizeof(int)));
  if (reset) {
    const int z[4] = {0, 0, 0, 0};
    CAPGEN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sk_diag), z, sizeof(z)));
  }
}

// the persisted autotune table: $CAPGEN_TUNE_TABLE, else tune_gfx950.txt next to libcapgen.so
// ("0" or "": none), loaded once per process before the first GEMM
static void load_default_tune_table() {
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("CAPGEN_TUNE_TABLE");
    std::string path;
    if (e) {
      if (!e[0] || (e[0] == '0' && !e[1])) return;
      path = e;
    } else {
      Dl_info info;
      if (!dladdr((void*)&gemm_init, &info) || !info.dli_fname) return;
      path = info.dli_fname;
      const size_t slash = path.rfind('/');
      path = (slash == std::string::npos ? std::string(".") : path.substr(0, slash)) + "/tune_gfx950.txt";
    }
    const int n = gemm_tune_load(path.c_str());
    if (knob(Knob::AutotuneLog)) std::fprintf(stderr, "[capgen gemm] tune table %s: %d entries\n", path.c_str(), n);
  });
}

void gemm_init() {
  load_default_tune_table();
  g_splitk_proto = knob(Knob::SplitkProto);
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  require(dev >= 0 && dev < 64, "gemm_init: device index out of range");
  if (!g_zero_page[dev]) {
    CAPGEN_HIP(hipMalloc(&g_zero_page[dev], 4096));
    CAPGEN_HIP(hipMemset(g_zero_page[dev], 0, 4096));
    CAPGEN_HIP(hipDeviceSynchronize());  // ordered before work on non-blocking streams
  }
}

void gemm_bf16(const GemmArgs& g_in, DType out, bool ta, bool tb, hipStream_t s) {
  GemmArgs g = g_in;
  if (g.wt < 0) g.wt = wt_default();
  if ((int64_t)g.M * g.ldc * (int64_t)dsize(out) >= (int64_t)0x7FFFFFFF) g.wt = 0;  // (32-bit buffer offsets)
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  require(g_zero_page[dev] != nullptr, "gemm: gemm_init() not called on this device");
  require(g.N % 4 == 0 && g.ldc % 4 == 0 && (g.aux == nullptr || g.ldaux % 4 == 0),
          "gemm(bf16): N/ldc must be multiples of 4");
  // read-modify-write epilogue: every 128-B line of C must belong to one tile (whole_lines)
  require(!g.beta || (((uintptr_t)g.C & 127) == 0 && (g.ldc * (int64_t)dsize(out)) % 128 == 0),
          "gemm(bf16): beta=1 needs C rows 128-B aligned (one writer per cache line)");
  require(!g.ce_stats || (out == DType::BF16 && !ta && !tb && !g.beta && !g.C2 && !g.aux && !g.relu && !g.colsum &&
                          g.ce_tgt && g.ce_tlogit && g.ce_ld >= (g.N + 15) / 16),
          "gemm(bf16): the fused cross-entropy epilogue is a plain bf16 NT GEMM (+bias)");
  require(!g.dec_stats || (out == DType::F32 && !ta && !tb && !g.beta && !g.C2 && !g.aux && !g.relu && !g.colsum &&
                           !g.ce_stats && g.dec_ld >= (g.N + 15) / 16),
          "gemm(bf16): the decode slab-stats epilogue is a plain f32-out NT GEMM (+bias)");
  if (!ta && g.bt && gemm_breg_ok(g)) {  // B handed over as fragment pieces: the register-B kernel
    gemm_breg(g, out, s);
    return;
  }
  if (out == DType::F32) launch_bf16_layout<float>(g, ta, tb, s);
  else launch_bf16_layout<bf16>(g, ta, tb, s);
}

}  // namespace capgen
