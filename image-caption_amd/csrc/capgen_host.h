// capgen — host-only declarations shared by the device code and the host-only C++ (error type,
// run-time switches).  Includes no HIP header, so the host-only sources (layout.cpp, scst_host.cpp,
// tune_parse.cpp, knobs.cpp) also build with plain g++ (make asan).
#pragma once
#include <string>
#include <utility>

namespace capgen {

struct Error {
  std::string msg;
  explicit Error(std::string m) : msg(std::move(m)) {}
};

inline void require(bool ok, const std::string& what) {
  if (!ok) throw Error(what);
}

// ---- run-time switches (knobs.cpp) ----------------------------------------------------------
// Alternate implementations the parity tests compare, scheduling modes the hazard tests sweep and
// data-parallel options; defaults = the product path.  Process defaults from CAPGEN_<NAME> when the
// library first asks, capgen_set_knob afterwards; nothing on a launch path calls getenv.  The
// debug-only ones (garbage or racy results on purpose) exist only in the debug build (-DCAPGEN_DEBUG,
// libcapgen_debug.so): the product library keeps their defaults.
enum class Knob : int {
  FusedCe, GroupDw, FusedQkv, FusedAttnBwd, ColsumSide, DecodeCrossMfma, SlabDecode, DecodeGroupLds, AttnWave,
  CeVec8, BregDecode, DecodeLnFold, FusedBeamStep, OverlapFront, OverlapDec0, StripeClear, BucketBlocks, Zero, FwdGraph, FwdSplit, GenGraph, Streams,
  EventFence, DeferLoss, FrontJoin, Autotune, AutotuneLog,
  Skip, DebugDropJoin, SplitkProto, AllowPartialLines, DwVariant, HostTiming,  // debug build only
  Count
};
int knob(Knob k);
// 0 set (old value in *old), -1 unknown name, -2 a debug-only switch in the product library
int knob_set(const char* name, int value, int* old);
bool debug_build();

}  // namespace capgen
