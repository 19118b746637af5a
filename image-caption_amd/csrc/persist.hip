// capgen — persistent FFN pair, DEBUG BUILD ONLY (libcapgen_debug.so): the round-3/4 experiment kept
// as a fault-isolation target.  H = relu(X . W1^T + b1) and Y = H . W2^T (the
// encoder FFN, modules.py:96-110) as ONE launch whose workgroups pull tasks from an atomic queue:
// every W1 tile, then every W2 tile, which waits for its row block's W1 tiles (done[mt]).  Same tile
// code as the plain launches of variant 7 (gemm_tile.h, 64x64, 4 waves, 3 stages), so a correct run
// is bit-identical to them.  Round 4 measured every W2 tile wrong at every grid size, grid 1
// included, with H right; `mode` bits isolate where:
//   1  W2 tasks only (H from the plain W1 launch; the host pre-sets done[] = tn1)
//   2  the W2 tile gets a private copy of its GemmArgs (not a reference into the kernel argument)
//   4  no consumer acquire
//   16 no task loop: one W2 tile per workgroup (blockIdx), the same FfnTask argument
//   32 no task loop, the kernel argument is the W2 GemmArgs alone
//   64 the task loop compiled without the W1 branch (W2 tasks only, as bit 1)
//   128 one gemm_tile call site for both GEMMs (the task selects its GemmArgs)
//   256 the round-4 loop shape (ffn_persist_r4_kernel)
// Not in the product library (the body compiles only with -DCAPGEN_DEBUG); not in include/capgen.h.
#include <cstdio>
#include <vector>

#include "gemm_tile.h"

namespace capgen {

#ifdef CAPGEN_DEBUG
namespace {

constexpr int PBM = 64, PBN = 64, PWM = 2, PWN = 2, PST = 3;
typedef TileCfg<false, false, PBM, PBN, PWM, PWN, PST> PCfg;
constexpr uint64_t kDeadlineTicks = 200000000ull;  // s_memrealtime runs at 100 MHz: 2 s per launch

struct FfnTask {
  GemmArgs g1, g2;
  int tm, tn1, tn2, mode;
  int* done;   // [tm] W1 tiles finished per row block
  int* queue;  // [0] next task, [1] workgroups finished, [2] give-ups
};

__device__ __forceinline__ int wave_fetch_add1(int* p, int v) {
  const int lane = __lane_id();
  const int old = __hip_atomic_fetch_add(p, lane == 0 ? v : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane(old);
}

__global__ void __launch_bounds__(256) ffn_w2_direct_kernel(FfnTask p) {
  __shared__ __attribute__((aligned(1024))) char smem[PCfg::SMEM];
  const int u = blockIdx.x, mt = u / p.tn2, nt = u % p.tn2;
  gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(p.g2, mt, nt, u, 0, 1, nullptr, nullptr, nullptr, smem);
}
__global__ void __launch_bounds__(256) ffn_w2_args_kernel(GemmArgs g, int tn2) {
  __shared__ __attribute__((aligned(1024))) char smem[PCfg::SMEM];
  const int u = blockIdx.x, mt = u / tn2, nt = u % tn2;
  gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(g, mt, nt, u, 0, 1, nullptr, nullptr, nullptr, smem);
}

template <bool W1, bool ONE_SITE>
__global__ void __launch_bounds__(256) ffn_persist_kernel(FfnTask p) {
  __shared__ __attribute__((aligned(1024))) char smem[PCfg::SMEM];
  __shared__ int s_task;
  const int n1 = p.tm * p.tn1, total = n1 + p.tm * p.tn2;
  const int first = (p.mode & 1) || !W1 ? n1 : 0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + kDeadlineTicks;
  for (;;) {
    if (wave == 0) {
      int t = total;
      if (__builtin_amdgcn_s_memrealtime() > deadline) (void)wave_fetch_add1(p.queue + 2, 1);
      else t = first + wave_fetch_add1(p.queue, 1);
      s_task = t;
    }
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    __syncthreads();
    if (t >= total) break;
    const bool w1 = W1 && t < n1;
    const int u = w1 ? t : t - n1, tn = w1 ? p.tn1 : p.tn2, mt = u / tn, nt = u % tn;
    if (!w1) {
      if (wave == 0) {
        while (wave_fetch_add1(p.done + mt, 0) < p.tn1) {
          __builtin_amdgcn_s_sleep(2);
          if (__builtin_amdgcn_s_memrealtime() > deadline) {
            (void)wave_fetch_add1(p.queue + 2, 1);
            break;
          }
        }
        if (!(p.mode & 4)) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __syncthreads();
    }
    if constexpr (ONE_SITE) {
      // one gemm_tile call site for both GEMMs: the task picks its arguments
      gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(w1 ? p.g1 : p.g2, mt, nt, u, 0, 1, nullptr, nullptr,
                                                             nullptr, smem);
    } else if (w1) {
      gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(p.g1, mt, nt, u, 0, 1, nullptr, nullptr, nullptr, smem);
    } else if (p.mode & 2) {
      GemmArgs g = p.g2;
      gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(g, mt, nt, u, 0, 1, nullptr, nullptr, nullptr, smem);
    } else {
      gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(p.g2, mt, nt, u, 0, 1, nullptr, nullptr, nullptr, smem);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave (and the next task's DMA waits)
    if (w1) {
      __syncthreads();
      if (wave == 0) (void)wave_fetch_add1(p.done + mt, 1);
    }
  }
}

// The round-4 shape of the task loop (two gemm_tile call sites in separate branches, each with its
// own barrier / counter code) -- kept to reproduce the wrong W2 tiles (mode bit 256)
__global__ void __launch_bounds__(256) ffn_persist_r4_kernel(FfnTask p) {
  __shared__ __attribute__((aligned(1024))) char smem[PCfg::SMEM];
  __shared__ int s_task;
  const int n1 = p.tm * p.tn1, total = n1 + p.tm * p.tn2;
  const int first = (p.mode & 1) ? n1 : 0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + kDeadlineTicks;
  for (;;) {
    if (wave == 0) {
      int t = total;
      if (__builtin_amdgcn_s_memrealtime() > deadline) (void)wave_fetch_add1(p.queue + 2, 1);
      else t = first + wave_fetch_add1(p.queue, 1);
      s_task = t;
    }
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    __syncthreads();
    if (t >= total) break;
    if (t < n1) {
      const int mt = t / p.tn1, nt = t % p.tn1;
      gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(p.g1, mt, nt, t, 0, 1, nullptr, nullptr, nullptr, smem);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (wave == 0) (void)wave_fetch_add1(p.done + mt, 1);
    } else {
      const int u = t - n1, mt = u / p.tn2, nt = u % p.tn2;
      if (wave == 0) {
        while (wave_fetch_add1(p.done + mt, 0) < p.tn1) {
          __builtin_amdgcn_s_sleep(2);
          if (__builtin_amdgcn_s_memrealtime() > deadline) {
            (void)wave_fetch_add1(p.queue + 2, 1);
            break;
          }
        }
        if (!(p.mode & 4)) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __syncthreads();
      gemm_tile<bf16, false, false, PBM, PBN, PWM, PWN, PST>(p.g2, mt, nt, u, 0, 1, nullptr, nullptr, nullptr, smem);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
}

__global__ void init_counters_kernel(int* buf, int tm, int done_val) {
  for (int i = threadIdx.x; i < 4 + tm; i += blockDim.x) buf[i] = i < 4 ? 0 : done_val;
}

int* g_pbuf[64] = {};
int g_pcap[64] = {};

}  // namespace
#endif  // CAPGEN_DEBUG

}  // namespace capgen

#ifdef CAPGEN_DEBUG
// Debug-build export (no declaration in include/capgen.h; tools/persist_ffn.py binds it): 0 = ran,
// -2 = bad arguments, -3 = a HIP error.  giveups != null: synchronises and returns the bounded waits
// that expired (0 when correct); null: fully asynchronous (graph-capturable).
extern "C" int capgen_dbg_ffn_persist(int M, int d, int fe, const void* X, const void* W1, const float* b1,
                                      const void* W2, void* H, void* Y, int grid, int mode, int* giveups,
                                      void* stream) {
  using namespace capgen;
  if (M <= 0 || fe % 64 || d % 64 || grid < 1 || grid > 4096 || !X || !W1 || !W2 || !H || !Y) return -2;
  try {
    hipStream_t s = (hipStream_t)stream;
    gemm_init();
    int dev = 0;
    CAPGEN_HIP(hipGetDevice(&dev));
    FfnTask p;
    p.g1.M = M, p.g1.N = fe, p.g1.K = d, p.g1.A = X, p.g1.lda = d, p.g1.B = W1, p.g1.ldb = d, p.g1.C = H;
    p.g1.ldc = fe, p.g1.bias = b1, p.g1.relu = 1, p.g1.wt = 1;
    p.g2.M = M, p.g2.N = d, p.g2.K = fe, p.g2.A = H, p.g2.lda = fe, p.g2.B = W2, p.g2.ldb = fe, p.g2.C = Y;
    p.g2.ldc = d, p.g2.wt = 0;
    p.tm = (M + PBM - 1) / PBM, p.tn1 = fe / PBN, p.tn2 = d / PBN, p.mode = mode;
    if (g_pcap[dev] < 4 + p.tm) {
      if (g_pbuf[dev]) CAPGEN_HIP(hipFree(g_pbuf[dev]));
      g_pcap[dev] = 4 + p.tm;
      CAPGEN_HIP(hipMalloc(&g_pbuf[dev], g_pcap[dev] * sizeof(int)));
    }
    // counters: queue / finished / give-ups zero, done[] zero (or tn1 when W2 runs alone), all on the
    // stream (graph-capturable; no host synchronisation unless the give-ups are read back)
    p.queue = g_pbuf[dev], p.done = g_pbuf[dev] + 4;
    init_counters_kernel<<<1, 256, 0, s>>>(g_pbuf[dev], p.tm, (mode & (1 | 64)) ? p.tn1 : 0);
    if (mode & 16) ffn_w2_direct_kernel<<<p.tm * p.tn2, 256, 0, s>>>(p);
    else if (mode & 32) ffn_w2_args_kernel<<<p.tm * p.tn2, 256, 0, s>>>(p.g2, p.tn2);
    else if (mode & 64) ffn_persist_kernel<false, false><<<grid, 256, 0, s>>>(p);
    else if (mode & 128) ffn_persist_kernel<true, true><<<grid, 256, 0, s>>>(p);
    else if (mode & 256) ffn_persist_r4_kernel<<<grid, 256, 0, s>>>(p);
    else ffn_persist_kernel<true, false><<<grid, 256, 0, s>>>(p);
    CAPGEN_HIP(hipGetLastError());
    if (!giveups) return 0;
    int gv = 0;
    CAPGEN_HIP(hipMemcpyAsync(&gv, g_pbuf[dev] + 2, sizeof(int), hipMemcpyDeviceToHost, s));
    CAPGEN_HIP(hipStreamSynchronize(s));
    if (giveups) *giveups = gv;
    return 0;
  } catch (const Error& e) {
    std::fprintf(stderr, "capgen_dbg_ffn_persist: %s\n", e.msg.c_str());
    return -3;
  }
}
#endif  // CAPGEN_DEBUG
