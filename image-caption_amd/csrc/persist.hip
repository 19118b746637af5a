// capgen — persistent FFN sub-block (experiment for the "fewer dependent kernel boundaries" lever):
// H = relu(X . W1^T + b1) and Y = H . W2^T in ONE launch, the encoder FFN of modules.py:96-110
// (PositionwiseFeedForward) at C2: 2304 x 2048 x 512 then 2304 x 512 x 2048.
//
// A grid of G workgroups (256 threads, 48 KB LDS each) pulls tasks from one atomic queue in
// dependency order: every W1 tile (row block by row block), then every W2 tile.  A W2 tile of row
// block mt needs the whole H row block (all fe/64 W1 column tiles of mt), so each W1 tile counts
// itself into done[mt]; a W2 task waits for that count.  Every task a workgroup waits on was
// dequeued before it (by a running workgroup), so the wait always ends.
//
// Hand-off (MI355X_MICROARCH.md 'Valid forms'): the producer stores its H tile write-through
// (GemmArgs::wt, sc1 buffer stores), every storing wave waits vmcnt(0), the workgroup barrier, one
// wave adds 1 to done[mt] (relaxed, agent scope).  The consumer's wave 0 polls, runs ONE agent acquire
// + vmcnt(0), then the barrier before any wave's operand DMA.  Every wait is bounded in time (a
// give-up count into queue[2]); the last workgroup to finish re-arms the counters for the next launch.
//
// The round-3 hang (one workgroup on one row block never returned) was control flow, not the
// hand-off.  The task index was read back from LDS through a generic `volatile int*`, so hipcc took
// it for a per-lane value, and lane 0 alone ran the queue atomic (`if (threadIdx.x == 0)`) at the top
// of the loop and the done[] add at the end of a W1 task.  hipcc threaded that loop-invariant lane
// condition into a nested loop (ISA of the old kernel, `hipcc --cuda-device-only -S`: the
// global_atomic_add sat in the outer loop; the barrier pair, the flat_load of the slot and the W1
// tile in an inner loop whose exit mask was `threadIdx.x == 0`).  Under SIMT exec masking, lanes 1-63
// of wave 0 and waves 1-3 kept cycling through the inner loop -- re-reading the unchanged slot and
// re-running the same tile -- while lane 0 waited for them to leave it: a livelock, with or without
// other workgroups.  Now every branch is on a wave-uniform (SGPR) value: the task index goes through
// readfirstlane, and the single-lane atomics became whole-wave calls of wave_fetch_add1 under
// `wave == 0`.  In the new ISA every branch of the task loop is an scc/vcc branch on SGPR values: waves
// 1-3 skip wave 0's atomic block as a whole, and every wave runs the same barriers per task.
// Same tile code (gemm_tile.h, 64x64, 4 waves, 3 stages) and k order as the plain launches of that
// variant, so the outputs are bit-identical to them (tools/persist_ffn.py checks and times both).
#include "gemm_tile.h"
#include "persist.h"

namespace capgen {
namespace {

constexpr int PBM = 64, PBN = 64, PWM = 2, PWN = 2, PST = 3;
typedef TileCfg<false, false, PBM, PBN, PWM, PWN, PST> PCfg;
constexpr uint64_t kDeadlineTicks = 200000000ull;  // s_memrealtime runs at 100 MHz: 2 s per launch

struct FfnTask {
  GemmArgs g1, g2;  // W1 (bias + relu, H write-through) and W2
  int tm, tn1, tn2;  // row blocks, W1 / W2 column tiles
  int* done;         // [tm] W1 tiles finished per row block
  int* queue;        // [0] next task, [1] workgroups finished, [2] give-ups
  int acquire;       // diagnostic: 0 drops the consumer acquire
};

// one atomic per wave, no single-lane branch: every lane of the (wave-uniform) caller adds `lane == 0`,
// hipcc's atomic optimizer folds that into ONE add of 1, and lane 0's old value is broadcast
__device__ __forceinline__ int wave_fetch_add1(int* p, int v) {
  const int lane = __lane_id();
  const int old = __hip_atomic_fetch_add(p, lane == 0 ? v : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane(old);
}

__global__ void __launch_bounds__(256) ffn_persist_kernel(FfnTask p) {
  __shared__ __attribute__((aligned(1024))) char smem[PCfg::SMEM];
  __shared__ int s_task;
  const int n1 = p.tm * p.tn1, total = n1 + p.tm * p.tn2;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + kDeadlineTicks;
  // Control flow is wave-uniform throughout (branches on SGPR values only): a single-lane branch
  // (`if (threadIdx.x == 0)`) at both ends of the loop body let hipcc thread the loop-invariant lane
  // condition into a nested loop that separates lane 0 from the barriers (see the header).
  for (;;) {
    if (wave == 0) {
      // past the deadline the queue is drained without work (results wrong, counted as a give-up)
      int t = total;
      if (__builtin_amdgcn_s_memrealtime() > deadline) (void)wave_fetch_add1(p.queue + 2, 1);
      else t = wave_fetch_add1(p.queue, 1);
      s_task = t;
    }
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    __syncthreads();  // every wave has read the slot before wave 0 may refill it
    if (t >= total) break;
    if (t < n1) {
      const int mt = t / p.tn1, nt = t % p.tn1;
      gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(p.g1, mt, nt, t, 0, 1, nullptr, nullptr, nullptr, smem);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
      __syncthreads();
      if (wave == 0) (void)wave_fetch_add1(p.done + mt, 1);
    } else {
      const int u = t - n1, mt = u / p.tn2, nt = u % p.tn2;
      if (wave == 0) {
        // the poll is an atomic read-modify-write (+0): a plain or sc1 load is served from this XCD's
        // L2, which measured never seeing the other XCDs' adds here (every wait gave up)
        while (wave_fetch_add1(p.done + mt, 0) < p.tn1) {
          __builtin_amdgcn_s_sleep(2);
          if (__builtin_amdgcn_s_memrealtime() > deadline) {  // bounded: give up (results wrong, the grid drains)
            (void)wave_fetch_add1(p.queue + 2, 1);
            break;
          }
        }
        if (p.acquire) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // holds the barrier until the invalidate is done
        }
      }
      __syncthreads();
      gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(p.g2, mt, nt, u, 0, 1, nullptr, nullptr, nullptr, smem);
      // the next task's operand DMA starts with counted vmcnt waits that assume only its own loads
      // are in flight: drain this tile's epilogue stores first
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  if (wave == 0) {
    const int fin = wave_fetch_add1(p.queue + 1, 1);
    if (fin == (int)gridDim.x - 1 && __lane_id() == 0) {  // every other workgroup is past its last counter access
      for (int i = 0; i < p.tm; ++i) (void)__hip_atomic_exchange(p.done + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      (void)__hip_atomic_exchange(p.queue, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      (void)__hip_atomic_exchange(p.queue + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct PersistState {
  int* buf = nullptr;  // [0..3] queue, then done[]
  int cap = 0;
};
PersistState g_ps[64];

}  // namespace

void ffn_persistent(const GemmArgs& g1, const GemmArgs& g2, int grid, int acquire, hipStream_t s) {
  require(g1.M == g2.M && g1.N == g2.K && g1.A && g1.B && g1.C && g2.B && g2.C && g2.A == g1.C,
          "ffn_persistent: W2 must read W1's output");
  require(g1.M > 0 && g1.N % PBN == 0 && g2.N % PBN == 0 && g1.K % 64 == 0 && g2.K % 64 == 0,
          "ffn_persistent: widths must be multiples of 64");
  require(g1.lda % 8 == 0 && g1.ldb % 8 == 0 && g1.ldc % 8 == 0 && g2.ldb % 8 == 0 && g2.ldc % 8 == 0,
          "ffn_persistent: 16-B aligned rows");
  require(grid >= 1 && grid <= 4096, "ffn_persistent: grid in [1, 4096]");
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  PersistState& st = g_ps[dev];
  FfnTask p;
  p.g1 = g1, p.g2 = g2;
  p.g1.relu = 1, p.g1.wt = 1, p.g1.beta = 0, p.g2.beta = 0;
  if (p.g2.wt < 0) p.g2.wt = wt_default();
  p.tm = (g1.M + PBM - 1) / PBM, p.tn1 = g1.N / PBN, p.tn2 = g2.N / PBN;
  if (st.cap < 4 + p.tm) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    CAPGEN_HIP(hipStreamIsCapturing(s, &cs));
    require(cs == hipStreamCaptureStatusNone, "ffn_persistent: first call of a size must not be captured");
    if (st.buf) {
      CAPGEN_HIP(hipStreamSynchronize(s));  // an earlier launch may still read the old counters
      CAPGEN_HIP(hipFree(st.buf));
    }
    st.cap = 4 + p.tm;
    CAPGEN_HIP(hipMalloc(&st.buf, st.cap * sizeof(int)));
    // zeroed on the launch stream, so the first launch is ordered after it (a null-stream memset is
    // not ordered with a non-blocking stream)
    CAPGEN_HIP(hipMemsetAsync(st.buf, 0, st.cap * sizeof(int), s));
  }
  p.queue = st.buf, p.done = st.buf + 4, p.acquire = acquire;
  ffn_persist_kernel<<<grid, 256, 0, s>>>(p);
  CAPGEN_HIP(hipGetLastError());
}

int ffn_persistent_giveups(bool reset) {
  int dev = 0;
  CAPGEN_HIP(hipGetDevice(&dev));
  PersistState& st = g_ps[dev];
  if (!st.buf) return 0;
  CAPGEN_HIP(hipDeviceSynchronize());
  int v = 0;
  CAPGEN_HIP(hipMemcpy(&v, st.buf + 2, sizeof(int), hipMemcpyDeviceToHost));
  if (reset) CAPGEN_HIP(hipMemset(st.buf + 2, 0, sizeof(int)));
  if (reset) CAPGEN_HIP(hipDeviceSynchronize());
  return v;
}

}  // namespace capgen
