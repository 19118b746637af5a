// Kernel-boundary price vs the bytes a dependent chain hands from launch to launch (round 5): a chain of
// 200 launches, each reading the previous launch's output buffer (B bytes) and writing the next one
// (B bytes), 16-B accesses, 1024 workgroups of 256 threads, replayed as one hipGraph.  Stores plain
// (dirty in the writing XCD's L2 until the end-of-kernel release writes them back) or write-through
// (sc1: leave L2 as they are issued).  Prints us per launch; the streaming time of 2B bytes alone is
// (2B / ~5 TB/s).  The engine's chain hands 1.2-9.4 MB per boundary (bf16 activations at C2).
//   hipcc -O3 --offload-arch=gfx950 tools/boundary_bytes_probe.hip -o /tmp/bbp && /tmp/bbp
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      return 1;                                                          \
    }                                                                    \
  } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u4;

template <bool WT>
__global__ void __launch_bounds__(256) chain(const u4* __restrict__ in, u4* __restrict__ out, size_t n16) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7FFFFFFF, 0x00020000);
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    u4 v = in[i];
    v.x += 1u;
    if (WT) __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(i * 16), 0, 16 /* sc1 */);
    else out[i] = v;
  }
}

template <bool WT>
int run(hipStream_t s, u4* a, u4* b, size_t bytes) {
  const int n = 200;
  const size_t n16 = bytes / 16;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; ++i) chain<WT><<<1024, 256, 0, s>>>(i % 2 ? b : a, i % 2 ? a : b, n16);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::printf("bytes %9zu  %-13s  %6.2f us/launch\n", bytes, WT ? "write-through" : "plain", ms * 1e3 / (5 * n));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t maxb = 24u << 20;
  u4 *a, *b;
  CK(hipMalloc(&a, maxb));
  CK(hipMalloc(&b, maxb));
  CK(hipMemset(a, 0, maxb));
  CK(hipMemset(b, 0, maxb));
  for (size_t bytes : {(size_t)16384, (size_t)1u << 20, (size_t)2359296, (size_t)4718592, (size_t)9437184,
                       (size_t)24u << 20}) {
    if (run<false>(s, a, b, bytes)) return 1;
    if (run<true>(s, a, b, bytes)) return 1;
  }
  return 0;
}
