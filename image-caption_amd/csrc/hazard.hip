// capgen — cross-stream hazard checker + side-stream delay injection (see hazard.h).
#include "hazard.h"

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "capgen_common.h"

namespace capgen {
namespace hz {

namespace {

constexpr int kMaxStreams = 16;
typedef std::array<uint32_t, kMaxStreams> Clock;

void join(Clock& a, const Clock& b) {
  for (int i = 0; i < kMaxStreams; ++i) a[i] = std::max(a[i], b[i]);
}

struct Op {
  int stream;
  uint32_t seq;  // position on its stream (1-based)
  Clock vc;      // what the launch is ordered after
  const char* name;
  std::vector<Rgn> rg;
};

struct State {
  std::mutex mu;
  std::map<hipStream_t, int> sid;
  std::vector<Clock> sclk;
  std::map<hipEvent_t, Clock> eclk;
  Clock host{};
  std::vector<Op> ops;
  hipStream_t crit = nullptr;
  int idx(hipStream_t s) {
    auto it = sid.find(s);
    if (it != sid.end()) return it->second;
    require((int)sclk.size() < kMaxStreams, "hazard checker: too many streams");
    const int i = (int)sclk.size();
    sid[s] = i;
    sclk.push_back(Clock{});
    return i;
  }
};
State& st() {
  static State s;
  return s;
}

// spin on the 100 MHz real-time counter (a read of the clock; nothing is stored)
__global__ void hz_spin_kernel(int64_t ticks) {
  const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
  while ((int64_t)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}

bool env_on(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] && e[0] != '0';
}

bool overlap(const Rgn& a, const Rgn& b) {
  const uintptr_t alo = a.base, ahi = a.base + (a.rows - 1) * a.stride + a.bytes;
  const uintptr_t blo = b.base, bhi = b.base + (b.rows - 1) * b.stride + b.bytes;
  if (ahi <= blo || bhi <= alo) return false;
  if (a.rows == 1 && b.rows == 1) return true;
  if (a.rows > 1 && b.rows > 1) {
    if (a.stride != b.stride) return true;  // conservative
    const int64_t S = a.stride;
    const int64_t d = (((int64_t)(b.base - a.base)) % S + S) % S;  // b's column start in a's frame
    return d < a.bytes || d + b.bytes > S;
  }
  const Rgn& I = a.rows == 1 ? a : b;  // interval vs strided rows
  const Rgn& R = a.rows == 1 ? b : a;
  const int64_t lo = (int64_t)I.base - (int64_t)R.base, hi = lo + I.bytes;
  int64_t r = lo - R.bytes + 1 <= 0 ? 0 : (lo - R.bytes + 1 + R.stride - 1) / R.stride;  // first row ending past lo
  return r < R.rows && r * R.stride < hi;
}

const char* kname(int k) { return k == WR ? "write" : k == ACC ? "accumulate" : "read"; }

}  // namespace

bool g_log = env_on("CAPGEN_HAZARD");
int64_t g_delay = [] {  // (debug build: CAPGEN_SIDE_DELAY microseconds; set_side_delay in any build)
  const char* e = debug_build() ? std::getenv("CAPGEN_SIDE_DELAY") : nullptr;
  return e ? (int64_t)(std::atof(e) * 100.0) : (int64_t)0;
}();

void enable(bool log) {
  State& S = st();
  std::lock_guard<std::mutex> lk(S.mu);
  g_log = log;
}
void set_delay_us(double us) { g_delay = us > 0 ? (int64_t)(us * 100.0) : 0; }
void set_critical(hipStream_t s) { st().crit = s; }

void reset() {
  State& S = st();
  std::lock_guard<std::mutex> lk(S.mu);
  S.ops.clear();
  S.eclk.clear();
  for (auto& c : S.sclk) c = Clock{};
  S.host = Clock{};
}

int64_t log_size() { return (int64_t)st().ops.size(); }

void op(hipStream_t s, const char* name, const Rgn* rgns, size_t n) {
  State& S = st();
  if (g_delay > 0 && s != S.crit) {
    hz_spin_kernel<<<1, 64, 0, s>>>(g_delay);
    CAPGEN_HIP(hipGetLastError());
  }
  if (!g_log) return;
  std::lock_guard<std::mutex> lk(S.mu);
  const int i = S.idx(s);
  Clock& c = S.sclk[i];
  join(c, S.host);
  ++c[i];
  Op o;
  o.stream = i, o.seq = c[i], o.vc = c, o.name = name;
  for (size_t k = 0; k < n; ++k)
    if (rgns[k].rows > 0 && rgns[k].bytes > 0) o.rg.push_back(rgns[k]);
  S.ops.push_back(std::move(o));
}

void record(hipEvent_t e, hipStream_t s) {
  CAPGEN_HIP(hipEventRecord(e, s));
  if (!g_log) return;
  State& S = st();
  std::lock_guard<std::mutex> lk(S.mu);
  Clock& c = S.sclk[S.idx(s)];
  join(c, S.host);
  S.eclk[e] = c;
}

void wait(hipStream_t s, hipEvent_t e) {
  CAPGEN_HIP(hipStreamWaitEvent(s, e, 0));
  if (!g_log) return;
  State& S = st();
  std::lock_guard<std::mutex> lk(S.mu);
  auto it = S.eclk.find(e);
  if (it == S.eclk.end()) return;  // never recorded (in this log): no edge
  join(S.sclk[S.idx(s)], it->second);
}

void host_sync(hipStream_t s) {
  if (s) CAPGEN_HIP(hipStreamSynchronize(s));
  else CAPGEN_HIP(hipDeviceSynchronize());
  if (!g_log) return;
  State& S = st();
  std::lock_guard<std::mutex> lk(S.mu);
  if (s) {
    join(S.host, S.sclk[S.idx(s)]);
  } else {
    for (auto& c : S.sclk) join(S.host, c);
  }
}

int check(std::string* report, int max_lines) {
  State& S = st();
  std::lock_guard<std::mutex> lk(S.mu);
  int n = 0;
  std::map<std::string, int> seen;  // one report line per (kernel pair, kinds)
  for (size_t j = 0; j < S.ops.size(); ++j) {
    const Op& B = S.ops[j];
    for (size_t i = 0; i < j; ++i) {
      const Op& A = S.ops[i];
      if (A.stream == B.stream || B.vc[A.stream] >= A.seq) continue;  // same stream / ordered
      for (const Rgn& ra : A.rg) {
        bool hit = false;
        for (const Rgn& rb : B.rg) {
          if ((ra.kind == RD && rb.kind == RD) || (ra.kind == ACC && rb.kind == ACC)) continue;
          if (!overlap(ra, rb)) continue;
          ++n;
          hit = true;
          if (report) {
            char key[256];
            std::snprintf(key, sizeof key, "%s(%s, stream %d) <-> %s(%s, stream %d)", A.name, kname(ra.kind), A.stream,
                          B.name, kname(rb.kind), B.stream);
            if (seen[key]++ == 0 && (int)seen.size() <= max_lines) {
              char line[400];
              std::snprintf(line, sizeof line, "launch %zu %s  vs  launch %zu: bytes [%#lx, +%ld) / [%#lx, +%ld)\n", i,
                            key, j, (unsigned long)ra.base, (long)((ra.rows - 1) * ra.stride + ra.bytes),
                            (unsigned long)rb.base, (long)((rb.rows - 1) * rb.stride + rb.bytes));
              *report += line;
            }
          }
          break;
        }
        if (hit) break;
      }
    }
  }
  return n;
}

}  // namespace hz
}  // namespace capgen
