// Launch-overhead probe for MI355X: what does one dependent kernel boundary cost on this
// stack (ROCm 7, eager vs hipGraph, one stream vs an event fork/join to a second stream)?
// Build: hipcc -O3 --offload-arch=gfx950 tools/kprobe.hip -o tools/kprobe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <functional>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));         \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

__global__ void tiny(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f;
}
// streaming copy, 16 B per lane
__global__ void copyk(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

static float time_it(hipStream_t s, int reps, const std::function<void()>& f) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / reps;
}

int main() {
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ef, ej;
  CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
  float* p;
  CK(hipMalloc(&p, 1 << 20));
  const size_t nbytes = 1216 * 512 * 2 * 2;  // ~2.5 MB (an LN-sized read+write)
  float4 *a, *b;
  CK(hipMalloc(&a, nbytes));
  CK(hipMalloc(&b, nbytes));
  CK(hipMemset(a, 0, nbytes));
  const int K = 200;
  auto chain = [&](int grid, bool fork) {
    for (int i = 0; i < K; ++i) {
      tiny<<<grid, 256, 0, s>>>(p);
      if (fork) {
        CK(hipEventRecord(ef, s));
        CK(hipStreamWaitEvent(s2, ef, 0));
        tiny<<<grid, 256, 0, s2>>>(p + 64);
        CK(hipEventRecord(ej, s2));
        CK(hipStreamWaitEvent(s, ej, 0));
      }
    }
  };
  auto copies = [&]() {
    for (int i = 0; i < K; ++i) copyk<<<1024, 256, 0, s>>>(a, b, nbytes / 16);
  };
  std::printf("eager tiny 1 WG       : %.2f us/kernel\n", time_it(s, 3, [&] { chain(1, false); }) / K);
  std::printf("eager tiny 1024 WG    : %.2f us/kernel\n", time_it(s, 3, [&] { chain(1024, false); }) / K);
  std::printf("eager copy 2.5MB      : %.2f us/kernel\n", time_it(s, 3, copies) / K);
  std::printf("eager fork/join pair  : %.2f us/iter (2 kernels + 2 events)\n",
              time_it(s, 3, [&] { chain(1024, true); }) / K);
  // graphs
  auto graph_of = [&](const std::function<void()>& f) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    f();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    return ge;
  };
  hipGraphExec_t g1 = graph_of([&] { chain(1024, false); });
  hipGraphExec_t g2 = graph_of(copies);
  hipGraphExec_t g3 = graph_of([&] { chain(1024, true); });
  std::printf("graph tiny 1024 WG    : %.2f us/kernel\n", time_it(s, 3, [&] { CK(hipGraphLaunch(g1, s)); }) / K);
  std::printf("graph copy 2.5MB      : %.2f us/kernel\n", time_it(s, 3, [&] { CK(hipGraphLaunch(g2, s)); }) / K);
  std::printf("graph fork/join pair  : %.2f us/iter\n", time_it(s, 3, [&] { CK(hipGraphLaunch(g3, s)); }) / K);
  // two independent chains in ONE graph (fork at the start, join at the end): is a 2-branch
  // graph launched as cheaply as a linear one?
  {
    auto two = [&]() {
      CK(hipEventRecord(ef, s));
      CK(hipStreamWaitEvent(s2, ef, 0));
      for (int i = 0; i < K; ++i) {
        tiny<<<1024, 256, 0, s>>>(p);
        tiny<<<1024, 256, 0, s2>>>(p + 64);
      }
      CK(hipEventRecord(ej, s2));
      CK(hipStreamWaitEvent(s, ej, 0));
    };
    hipGraphExec_t g4 = graph_of(two);
    std::printf("graph 2 chains        : %.2f us/kernel-pair\n", time_it(s, 3, [&] { CK(hipGraphLaunch(g4, s)); }) / K);
    CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::high_resolution_clock::now();
    CK(hipGraphLaunch(g4, s));
    auto t1 = std::chrono::high_resolution_clock::now();
    CK(hipStreamSynchronize(s));
    std::printf("host graph 2 chains   : %.2f us/kernel-pair\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / K);
    t0 = std::chrono::high_resolution_clock::now();
    CK(hipGraphLaunch(g1, s));
    t1 = std::chrono::high_resolution_clock::now();
    CK(hipStreamSynchronize(s));
    std::printf("host graph 1 chain    : %.2f us/kernel\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / K);
    t0 = std::chrono::high_resolution_clock::now();
    two();
    t1 = std::chrono::high_resolution_clock::now();
    CK(hipStreamSynchronize(s));
    std::printf("host eager 2 chains   : %.2f us/kernel-pair\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / K);
  }
  // host enqueue rate
  {
    auto t0 = std::chrono::high_resolution_clock::now();
    chain(1024, false);
    auto t1 = std::chrono::high_resolution_clock::now();
    CK(hipStreamSynchronize(s));
    std::printf("host enqueue          : %.2f us/kernel\n",
                std::chrono::duration<double, std::micro>(t1 - t0).count() / K);
    t0 = std::chrono::high_resolution_clock::now();
    chain(1024, true);
    t1 = std::chrono::high_resolution_clock::now();
    CK(hipStreamSynchronize(s));
    std::printf("host enqueue fork/join: %.2f us/iter\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / K);
  }
  // what does a cross-stream signal cost the SIGNALLING stream? (no waits: a chain of 1024-WG
  // kernels on s with a marker after every kernel)
  {
    hipEvent_t eflag[3];
    const unsigned flags[3] = {hipEventDisableTiming, hipEventDisableTiming | hipEventReleaseToDevice,
                               hipEventDisableTiming | hipEventDisableSystemFence};
    const char* names[3] = {"default", "release-to-device", "no-system-fence"};
    for (int f = 0; f < 3; ++f) {
      CK(hipEventCreateWithFlags(&eflag[f], flags[f]));
      std::printf("eager kernel+record %-17s: %.2f us/iter\n", names[f], time_it(s, 3, [&] {
        for (int i = 0; i < K; ++i) {
          tiny<<<1024, 256, 0, s>>>(p);
          CK(hipEventRecord(eflag[f], s));
        }
      }) / K);
    }
    uint32_t* sig = nullptr;
    if (hipExtMallocWithFlags((void**)&sig, 4096, hipMallocSignalMemory) == hipSuccess) {
      std::printf("eager kernel+writeValue32        : %.2f us/iter\n", time_it(s, 3, [&] {
        for (int i = 0; i < K; ++i) {
          tiny<<<1024, 256, 0, s>>>(p);
          CK(hipStreamWriteValue32(s, sig, (uint32_t)i, 0));
        }
      }) / K);
      // a fork per kernel to a second stream (the engine's per-block flush): event record + wait vs
      // a memory write + a wait-on-value packet; the signalling stream's time per kernel
      hipEvent_t enf;
      CK(hipEventCreateWithFlags(&enf, hipEventDisableTiming | hipEventDisableSystemFence));
      std::printf("fork event (no system fence)     : %.2f us/iter\n", time_it(s, 3, [&] {
        for (int i = 0; i < K; ++i) {
          tiny<<<1024, 256, 0, s>>>(p);
          CK(hipEventRecord(enf, s));
          CK(hipStreamWaitEvent(s2, enf, 0));
          tiny<<<64, 256, 0, s2>>>(p + 64);
        }
      }) / K);
      CK(hipDeviceSynchronize());
      uint32_t seq = 1u << 20;
      std::printf("fork writeValue/waitValue        : %.2f us/iter\n", time_it(s, 3, [&] {
        for (int i = 0; i < K; ++i) {
          tiny<<<1024, 256, 0, s>>>(p);
          ++seq;
          CK(hipStreamWriteValue32(s, sig + 16, seq, 0));
          CK(hipStreamWaitValue32(s2, sig + 16, seq, hipStreamWaitValueGte, 0xFFFFFFFFu));
          tiny<<<64, 256, 0, s2>>>(p + 64);
        }
      }) / K);
      CK(hipDeviceSynchronize());
      std::printf("no fork (same kernels, s2 free)  : %.2f us/iter\n", time_it(s, 3, [&] {
        for (int i = 0; i < K; ++i) {
          tiny<<<1024, 256, 0, s>>>(p);
          tiny<<<64, 256, 0, s2>>>(p + 64);
        }
      }) / K);
      CK(hipDeviceSynchronize());
    } else {
      std::printf("signal memory unavailable\n");
    }
  }
  // host price of the runtime calls a launch wrapper tends to make
  auto host_us = [&](const char* what, const std::function<void()>& f) {
    const int R = 2000;
    f();
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < R; ++i) f();
    auto t1 = std::chrono::high_resolution_clock::now();
    std::printf("host %-22s: %.3f us/call\n", what, std::chrono::duration<double, std::micro>(t1 - t0).count() / R);
  };
  int dev;
  hipStreamCaptureStatus cst;
  host_us("hipGetDevice", [&] { (void)hipGetDevice(&dev); });
  host_us("hipGetLastError", [&] { (void)hipGetLastError(); });
  host_us("hipStreamIsCapturing", [&] { (void)hipStreamIsCapturing(s, &cst); });
  host_us("hipSetDevice", [&] { (void)hipSetDevice(0); });
  CK(hipStreamSynchronize(s));
  host_us("launch tiny (1 WG)", [&] { tiny<<<1, 64, 0, s>>>(p); });
  CK(hipStreamSynchronize(s));
  host_us("hipEventRecord", [&] { (void)hipEventRecord(ef, s); });
  CK(hipStreamSynchronize(s));
  host_us("hipStreamWaitEvent", [&] { (void)hipStreamWaitEvent(s2, ef, 0); });
  CK(hipDeviceSynchronize());
  return 0;
}
