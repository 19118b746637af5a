// capgen — the library's run-time switches (capgen_host.h `knob`).
//
// Every switch has a default that is the product path.  The CAPGEN_<NAME> environment variables set
// the process defaults once, when the library first asks; capgen_set_knob (tests: capgen._lib.set_knob)
// changes one afterwards.  Engines read the switches they keep when they are created, launch paths
// read the snapshot -- nothing on a launch path calls getenv.
//
// Debug-only switches make results garbage or racy on purpose (kernel-skip masks for marginal-cost
// probes, a dropped stream edge for the hazard checker's self-test, split-K hand-off protocol bits,
// forced GEMM variants): they exist only in the debug build (make debug -> libcapgen_debug.so,
// -DCAPGEN_DEBUG); the product library reads none of them and refuses to set them.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "capgen_host.h"

namespace capgen {
namespace {

struct KnobDef {
  Knob k;
  const char* name;  // CAPGEN_<name>
  int dflt;
  bool debug_only;
};

// (order = Knob order)
constexpr KnobDef kDefs[] = {
    // alternate implementations compared by the parity tests (1 = the product path)
    {Knob::FusedCe, "FUSED_CE", 1, false},                  // classifier + CE fused (0: f32 logits + ce_kernel)
    {Knob::GroupDw, "GROUP_DW", 1, false},                  // a block's weight gradients as one grouped launch
    {Knob::FusedQkv, "FUSED_QKV", 1, false},                // Q/K/V projection + attention in one launch
    {Knob::FusedAttnBwd, "FUSED_ATTN_BWD", 1, false},       // output-projection dX inside the attention backward
    {Knob::ColsumSide, "COLSUM_SIDE", 1, false},            // FFN bias sums on the weight-gradient stream
    {Knob::DecodeCrossMfma, "DECODE_CROSS_MFMA", 1, false},  // beam cross attention on the MFMA kernel
    {Knob::SlabDecode, "SLAB_DECODE", 1, false},            // decode selection from the slab stats
    {Knob::DecodeGroupLds, "DECODE_GROUP_LDS", 1, false},   // grouped decode attention stages K/V in LDS
    {Knob::AttnWave, "ATTN_WAVE", 1, false},                // one-wave attention forward for Lq <= 16
    {Knob::CeVec8, "CE_VEC8", 1, false},                    // ce_finish with 16-B accesses
    {Knob::BregDecode, "BREG_DECODE", 1, false},            // decode GEMMs on the register-B kernel
    {Knob::DecodeLnFold, "DECODE_LN_FOLD", 1, false},       // decode LayerNorms in the consumer GEMM (2: every site)
    {Knob::FusedBeamStep, "FUSED_BEAM_STEP", 1, false},     // beam selection + reorder in one launch per step
    // scheduling modes swept by the hazard tests / data-parallel options
    {Knob::OverlapFront, "OVERLAP_FRONT", 1, false},  // decoder front beside the encoder
    {Knob::OverlapDec0, "OVERLAP_DEC0", 1, false},    // decoder block 0 half beside the encoder backward
    {Knob::StripeClear, "STRIPE_CLEAR", 1, false},    // striped partial sums zeroed by their folds
    {Knob::BucketBlocks, "BUCKET_BLOCKS", 1, false},  // transformer blocks per gradient bucket
    {Knob::Zero, "ZERO", 1, false},                   // sharded update at world > 1 (2: also at world 1)
    {Knob::FwdGraph, "FWD_GRAPH", 1, false},          // forward replayed as one hipGraph at world 1 (2: at any world size)
    {Knob::FwdSplit, "FWD_SPLIT", 0, false},          // split forward graphs
    {Knob::GenGraph, "GEN_GRAPH", 0, false},          // decode steps as captured graphs
    {Knob::Streams, "STREAMS", 3, false},             // engine streams (3, 2 or 1)
    {Knob::EventFence, "EVENT_FENCE", 1, false},      // 1 no system fence, 2 device release, 0 HIP default
    {Knob::DeferLoss, "DEFER_LOSS", 1, false},        // train step's loss mean on es2 (0: on the critical stream)
    {Knob::FrontJoin, "FRONT_JOIN", 99, false},       // forward joins the decoder front before encoder block N (> Le: before the decoder)
    {Knob::Autotune, "AUTOTUNE", 1, false},           // time GEMM shapes the tune table lacks
    {Knob::AutotuneLog, "AUTOTUNE_LOG", 0, false},    // print tuning decisions
    // debug build only
    {Knob::Skip, "SKIP", 0, true},                             // kernel classes to skip (marginal-cost probes)
    {Knob::DebugDropJoin, "DEBUG_DROP_JOIN", 0, true},         // drop the side-stream join (checker self-test)
    {Knob::SplitkProto, "SPLITK_PROTO", 0, true},              // split-K hand-off protocol bits
    {Knob::AllowPartialLines, "ALLOW_PARTIAL_LINES", 0, true},  // GEMM tiles narrower than a 128-B line
    {Knob::DwVariant, "DW_VARIANT", 0, true},                  // weight-gradient GEMMs on a fixed variant
    {Knob::HostTiming, "HOST_TIMING", 0, true},                // print host enqueue times
};
static_assert(sizeof(kDefs) / sizeof(kDefs[0]) == (size_t)Knob::Count, "one definition per knob");

#ifdef CAPGEN_DEBUG
constexpr bool kDebugBuild = true;
#else
constexpr bool kDebugBuild = false;
#endif

std::atomic<int> g_val[(int)Knob::Count];
std::once_flag g_once;

void init() {
  for (const KnobDef& d : kDefs) {
    int v = d.dflt;
    if (!d.debug_only || kDebugBuild) {
      const std::string env = std::string("CAPGEN_") + d.name;
      if (const char* e = std::getenv(env.c_str())) v = std::atoi(e);
    }
    g_val[(int)d.k].store(v, std::memory_order_relaxed);
  }
}

}  // namespace

int knob(Knob k) {
  std::call_once(g_once, init);
  return g_val[(int)k].load(std::memory_order_relaxed);
}

int knob_set(const char* name, int value, int* old) {
  std::call_once(g_once, init);
  for (const KnobDef& d : kDefs)
    if (std::strcmp(d.name, name) == 0) {
      if (d.debug_only && !kDebugBuild) return -2;
      const int prev = g_val[(int)d.k].exchange(value, std::memory_order_relaxed);
      if (old) *old = prev;
      return 0;
    }
  return -1;
}

bool debug_build() { return kDebugBuild; }

}  // namespace capgen
