// XCD-local phase barrier vs kernel boundary (round 6, VERDICT r5 item 1's first step): what does one
// phase seam cost inside ONE persistent launch, where each group of 32 workgroups (blockIdx % 8: one
// XCD under round-robin dispatch -- speed only, never correctness) meets at a counter barrier, against
// the same phase as its own launch in a hipGraph-replayed chain?
//
// Every phase, every workgroup (256 threads, 256 workgroups = one per CU) reads R bytes of its GROUP's
// output of the previous phase (the other 31 workgroups' slabs, as a GEMM phase reads the group's
// activation rows) and writes W bytes of its own slab.  Forms:
//   chain     one launch per phase (plain stores), replayed as one graph: the engine's form today
//   wt        one launch, all phases: payload stored write-through (sc1) and read with sc1 loads, each
//             storing wave drains (vmcnt(0)), barrier, lane 0 adds to the group counter (agent scope),
//             one wave polls it relaxed with s_sleep, barrier -- no fence (MI355X_MICROARCH.md § visibility,
//             Valid forms, first table row)
//   fence     the same with plain stores, lane-0 release fence before the add and an acquire fence after
//             the poll, plain loads (Guideline 16's plain form)
// With --side a streaming kernel (one 256-thread workgroup per CU, 16-B loads and stores over 2 x 512 MB,
// the shape of the step's bucket Adam) runs on a second stream over the whole timed region: the seams
// then pay the contention the engine's critical chain sees from its side streams.
// Prints us per phase (time of the form / phases).  Every spin is bounded (timeout word -> exit).
//   hipcc -O3 --offload-arch=gfx950 tools/xcd_phase_probe.hip -o tools/xcd_phase_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u4;
typedef __attribute__((address_space(1))) unsigned int gu32;

constexpr int NWG = 256, GROUPS = 8, PER = NWG / GROUPS;

// slab of workgroup w: buf + w * slab_stride (bytes); R bytes read = the group's slabs in turn
__device__ __forceinline__ u4 body_read(const char* buf, size_t slab, int g, int R, bool sc1,
                                        __amdgpu_buffer_rsrc_t rin) {
  u4 acc = {0u, 0u, 0u, 0u};
  // the R bytes: 16 B per lane per step, walking the group's 32 slabs (w = g + 8 j)
  const int per = (int)(slab / 16);  // 16-B pieces per slab
  for (int i = threadIdx.x; i < R / 16; i += 256) {
    const int j = (i / per) % PER, o = i % per;
    const unsigned off = (unsigned)(((size_t)(g + GROUPS * j) * slab) + (size_t)o * 16);
    u4 v = sc1 ? __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 16)
               : *reinterpret_cast<const u4*>(buf + off);
    acc += v;
  }
  return acc;
}

__device__ __forceinline__ void body_write(char* buf, size_t slab, int w, int W, u4 acc, bool sc1,
                                           __amdgpu_buffer_rsrc_t rout) {
  for (int i = threadIdx.x; i < W / 16; i += 256) {
    const unsigned off = (unsigned)((size_t)w * slab + (size_t)i * 16);
    u4 v = acc;
    v.x += (unsigned)i;
    if (sc1) __builtin_amdgcn_raw_buffer_store_b128(v, rout, off, 0, 16);
    else *reinterpret_cast<u4*>(buf + off) = v;
  }
}

__global__ void __launch_bounds__(256) phase_kernel(const char* in, char* out, size_t slab, int W, int R) {
  const int w = blockIdx.x, g = w % GROUPS;
  __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(in), 0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7FFFFFFF, 0x00020000);
  u4 acc = body_read(in, slab, g, R, false, rin);
  body_write(out, slab, w, W, acc, false, rout);
}

template <bool WT>
__global__ void __launch_bounds__(256) persistent_kernel(char* a, char* b, size_t slab, int W, int R, int nphase,
                                                         unsigned* ctr, unsigned* tmo) {
  const int w = blockIdx.x, g = w % GROUPS;
  __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(a, 0, 0x7FFFFFFF, 0x00020000);
  __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(b, 0, 0x7FFFFFFF, 0x00020000);
  gu32* c = (gu32*)(ctr + g * 32);  // one 128-B line per group
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  for (int ph = 0; ph < nphase; ++ph) {
    const bool odd = ph & 1;
    u4 acc = body_read(odd ? b : a, slab, g, R, WT, odd ? rb : ra);
    body_write(odd ? a : b, slab, w, W, acc, WT, odd ? ra : rb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its stores
    __syncthreads();
    if (threadIdx.x == 0) {
      if (!WT) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) {  // one wave polls
      const unsigned want = (unsigned)PER * (ph + 1);
      unsigned spins = 0;
      while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {  // bounded: record and leave (results garbage, time invalid)
          if (threadIdx.x == 0) atomicAdd(tmo, 1u), bad = 1;
          break;
        }
      }
      if (!WT && threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (bad) return;
  }
}

__global__ void __launch_bounds__(256) side_stream(const u4* __restrict__ x, u4* __restrict__ y, size_t n16, int reps) {
  for (int r = 0; r < reps; ++r)
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
      u4 v = __builtin_nontemporal_load(x + i);
      v.y += 1u;
      __builtin_nontemporal_store(v, y + i);
    }
}

int main(int argc, char** argv) {
  int W = 16384, R = 16384, nphase = 100, side = 0;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--side")) side = 1;
    else if (!std::strcmp(argv[i], "-W") && i + 1 < argc) W = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-R") && i + 1 < argc) R = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-n") && i + 1 < argc) nphase = std::atoi(argv[++i]);
  }
  const size_t slab = ((size_t)(W > R / PER ? W : R / PER) + 255) / 256 * 256;
  char *a, *b;
  unsigned *ctr, *tmo;
  CK(hipMalloc(&a, slab * NWG));
  CK(hipMalloc(&b, slab * NWG));
  CK(hipMemset(a, 0, slab * NWG));
  CK(hipMemset(b, 0, slab * NWG));
  CK(hipMalloc(&ctr, GROUPS * 128));
  CK(hipMalloc(&tmo, 16));
  CK(hipMemset(tmo, 0, 16));
  const size_t side_bytes = (size_t)512 << 20;
  u4 *sx = nullptr, *sy = nullptr;
  CK(hipMalloc(&sx, side_bytes));
  CK(hipMalloc(&sy, side_bytes));
  CK(hipMemset(sx, 0, side_bytes));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, es0, es1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&es0));
  CK(hipEventCreate(&es1));

  // graphs: the chain of nphase launches; each persistent form = memset of the counters + one launch
  hipGraphExec_t ex[3];
  for (int f = 0; f < 3; ++f) {
    hipGraph_t gr;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    if (f == 0) {
      for (int p = 0; p < nphase; ++p) phase_kernel<<<NWG, 256, 0, s>>>(p & 1 ? b : a, p & 1 ? a : b, slab, W, R);
    } else {
      CK(hipMemsetAsync(ctr, 0, GROUPS * 128, s));
      if (f == 1) persistent_kernel<true><<<NWG, 256, 0, s>>>(a, b, slab, W, R, nphase, ctr, tmo);
      else persistent_kernel<false><<<NWG, 256, 0, s>>>(a, b, slab, W, R, nphase, ctr, tmo);
    }
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ex[f], gr, nullptr, nullptr, 0));
    CK(hipGraphDestroy(gr));
  }
  const char* names[3] = {"chain (launch per phase)", "one launch, wt + counter", "one launch, fence + counter"};
  // the side stream's length: calibrate to ~2x the slowest form
  int reps = 1;
  float side_ms = 0;
  if (side) {
    CK(hipEventRecord(es0, s2));
    side_stream<<<256, 256, 0, s2>>>(sx, sy, side_bytes / 16, 1);
    CK(hipEventRecord(es1, s2));
    CK(hipEventSynchronize(es1));
    CK(hipEventElapsedTime(&side_ms, es0, es1));
  }
  std::printf("W %d B/workgroup written, R %d B read per phase, %d phases, side stream %s\n", W, R, nphase,
              side ? "on" : "off");
  for (int round = 0; round < 3; ++round)
    for (int f = 0; f < 3; ++f) {
      CK(hipGraphLaunch(ex[f], s));  // warm
      CK(hipStreamSynchronize(s));
      float best = 1e30f;
      for (int it = 0; it < 5; ++it) {
        if (side) {
          reps = (int)(3.0f * 0.02f * nphase / (side_ms > 0 ? side_ms : 1.f)) + 1;  // >= ~3x a 20 us/phase form
          side_stream<<<256, 256, 0, s2>>>(sx, sy, side_bytes / 16, reps);  // queued first, runs throughout
        }
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ex[f], s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipStreamSynchronize(s2));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      unsigned t = 0;
      CK(hipMemcpy(&t, tmo, 4, hipMemcpyDeviceToHost));
      std::printf("round %d  %-28s %7.2f us/phase%s\n", round, names[f], best * 1e3f / nphase,
                  t ? "  (TIMEOUT: invalid)" : "");
      if (t) return 2;
    }
  return 0;
}
