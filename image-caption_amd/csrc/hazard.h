// capgen — cross-stream hazard checker and side-stream delay injection (diagnostics).
//
// The engine issues every step on three HIP streams (critical path, weight gradients, gradient
// buckets) ordered only by events.  With CAPGEN_HAZARD=1 (or capgen_debug_hazard) every launch
// issued through the launchers (gemm, LayerNorm, attention, reductions, Adam, copies, memsets,
// RCCL calls) records its stream and the device byte ranges it reads, writes or accumulates into
// (atomic adds), and every event record / wait and host synchronisation records its edge.  The
// check builds happens-before from that log (vector clocks per stream; a wait joins the clock
// of the event's last record; a host sync joins the synchronised streams into every later
// issue) and reports every pair of launches on different streams that touch overlapping bytes,
// at least one of them writing (two accumulations commute), and are not ordered.
//
// CAPGEN_SIDE_DELAY=<us> (or capgen_debug_side_delay): a spin kernel of that length is issued in
// front of every launch that is NOT on the critical stream, so side-stream work lands late and
// any missing edge shows up as a result difference (deterministic delay injection).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <initializer_list>
#include <string>

namespace capgen {
namespace hz {

enum Kind : int { RD = 0, WR = 1, ACC = 2 };

// rows x row_bytes at base + r * stride (stride >= row_bytes; rows == 1: a plain interval)
struct Rgn {
  uintptr_t base = 0;
  int64_t rows = 0, bytes = 0, stride = 0;
  int kind = RD;
};
inline Rgn mk(const void* p, int64_t bytes, int kind) {
  Rgn r;
  r.base = (uintptr_t)p, r.rows = p && bytes > 0 ? 1 : 0, r.bytes = bytes, r.stride = bytes, r.kind = kind;
  return r;
}
inline Rgn rd(const void* p, int64_t bytes) { return mk(p, bytes, RD); }
inline Rgn wr(const void* p, int64_t bytes) { return mk(p, bytes, WR); }
inline Rgn acc(const void* p, int64_t bytes) { return mk(p, bytes, ACC); }
// a 2-D block: rows of row_bytes, `stride` bytes apart
inline Rgn blk(const void* p, int64_t rows, int64_t row_bytes, int64_t stride, int kind) {
  Rgn r;
  r.base = (uintptr_t)p, r.rows = p && rows > 0 && row_bytes > 0 ? rows : 0, r.bytes = row_bytes;
  r.stride = stride > row_bytes ? stride : row_bytes, r.kind = kind;
  return r;
}

extern bool g_log;       // logging on
extern int64_t g_delay;  // side-stream delay (cycles of the spin kernel), 0 = off
inline bool active() { return g_log || g_delay > 0; }

// one launch on stream s (name: kernel class, for the report)
void op(hipStream_t s, const char* name, const Rgn* rgns, size_t n);
inline void op(hipStream_t s, const char* name, std::initializer_list<Rgn> rgns) {
  op(s, name, rgns.begin(), rgns.size());
}
// rows of a [.., ld] activation covering batches 0..B-1 of L rows each, batch stride bs (elements)
inline Rgn rows_blk(const void* p, int B, int L, int64_t bs, int64_t ld, int64_t row_elems, int64_t esz, int kind) {
  const int64_t per = ld > 0 ? bs / ld : 0;
  const int64_t rows = B > 0 && L > 0 ? (int64_t)(B - 1) * per + L : 0;
  return blk(p, rows, row_elems * esz, ld * esz, kind);
}
// `s` records `e` / `s` waits for `e` (also issues the HIP call)
void record(hipEvent_t e, hipStream_t s);
void wait(hipStream_t s, hipEvent_t e);
// the host synchronised with stream s (nullptr: the whole device); also issues the HIP call
void host_sync(hipStream_t s);
// the critical stream of the running call (launches elsewhere get the injected delay)
void set_critical(hipStream_t s);

void enable(bool log);
void set_delay_us(double us);
void reset();
// number of unordered conflicting pairs in the log since reset(); report: the first few
int check(std::string* report, int max_lines = 20);
int64_t log_size();

}  // namespace hz
}  // namespace capgen
