// Kernel-boundary price on MI355X for the engine's launch shapes: a dependent chain of 200 launches
// of a trivial 256-workgroup kernel, by kernel-argument size (16 B .. 2.6 KB: GemmArgs ~300 B,
// GemmGroup ~2.6 KB), LDS footprint, and eager vs hipGraph replay.  Prints us per launch.
//   hipcc -O3 --offload-arch=gfx950 tools/boundary_probe.hip -o /tmp/boundary_probe && /tmp/boundary_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                            \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

template <int BYTES>
struct Args {
  float* out;
  char pad[BYTES - sizeof(float*)];
};

template <int BYTES, int LDS>
__global__ void __launch_bounds__(256) k(Args<BYTES> a) {
  __shared__ float sm[LDS / 4 > 0 ? LDS / 4 : 1];
  if (LDS > 0) {
    sm[threadIdx.x] = (float)a.pad[threadIdx.x % (BYTES - sizeof(float*))];
    __syncthreads();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) a.out[0] += (LDS > 0 ? sm[5] : 1.f);
}

__global__ void spin_kernel(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}

template <int BYTES, int LDS>
int run(hipStream_t s, float* out, int blocks, const char* name) {
  Args<BYTES> a{};
  a.out = out;
  const int n = 200;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) k<BYTES, LDS><<<blocks, 256, 0, s>>>(a);
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < n; ++i) k<BYTES, LDS><<<blocks, 256, 0, s>>>(a);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms_e = 0;
  CK(hipEventElapsedTime(&ms_e, e0, e1));
  // the same chain queued behind a 20 ms spin: the host is far ahead, so this is the GPU-side price
  spin_kernel<<<1, 64, 0, s>>>(20LL * 2100 * 1000);
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < n; ++i) k<BYTES, LDS><<<blocks, 256, 0, s>>>(a);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms_q = 0;
  CK(hipEventElapsedTime(&ms_q, e0, e1));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; ++i) k<BYTES, LDS><<<blocks, 256, 0, s>>>(a);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms_g = 0;
  CK(hipEventElapsedTime(&ms_g, e0, e1));
  std::printf("%-28s blocks %4d  eager %6.2f  eager-queued %6.2f  graph %6.2f us/launch\n", name, blocks,
              ms_e * 1e3 / n, ms_q * 1e3 / n, ms_g * 1e3 / (5 * n));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* out;
  CK(hipMalloc(&out, 64));
  CK(hipMemset(out, 0, 64));
  for (int blocks : {1, 256, 1024}) {
    if (run<16, 0>(s, out, blocks, "args 16 B")) return 1;
    if (run<320, 0>(s, out, blocks, "args 320 B")) return 1;
    if (run<2688, 0>(s, out, blocks, "args 2.6 KB")) return 1;
    if (run<320, 49152>(s, out, blocks, "args 320 B + 48 KB LDS")) return 1;
    if (run<320, 98304>(s, out, blocks, "args 320 B + 96 KB LDS")) return 1;
  }
  return 0;
}
