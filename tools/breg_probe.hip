// Input-gradient GEMM probe (round 5): dX[M,N] = dY[M,K] . W[K,N] (bf16, f32 accumulation) with the
// WEIGHT operand streamed straight into registers from a tiled copy -- the attention fronts' form
// (qkv_attn.hip) -- instead of through the LDS-DMA ring both operands take in gemm_tile.h.
//
// Why: the library's 64x64 NN tile ingests ~48 GB/s per CU in the step: its bytes in
// flight are capped by the LDS ring (3 x 16 KB at 4 stages), and its k-step phase waits on 16 LDS
// fragment reads per wave.  Here the weight fragments (private to a wave: waves split N) come as
// 1-KB coalesced pieces into a double-buffered register batch of QB 32-deep k-steps; only the
// activation rows (shared by the 4 waves) go through LDS.
//
// Tiled copy Bt: piece (j, ks) = 512 bf16; lane l holds W[32 ks + 8 (l >> 4) + e][16 j + (l & 15)],
// e = 0..7 (the B fragment of v_mfma_f32_16x16x32_bf16 for column block j, k-step ks).
//
// Prints per shape: us/launch of the probe kernel (200 launches, hipEvents), and its max relative
// error against a naive f32 GEMM.  Build: hipcc -O3 --offload-arch=gfx950 tools/breg_probe.hip -o tools/breg_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

__global__ void tile_t_kernel(const bf16* __restrict__ W, int K, int N, bf16* __restrict__ Bt) {
  // one thread per (piece, lane): 8 strided loads, one 16-B store
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int KS = K / 32;
  const int64_t pieces = (int64_t)(N / 16) * KS;
  if (i >= pieces * 64) return;
  const int lane = (int)(i & 63);
  const int64_t p = i >> 6;
  const int j = (int)(p / KS), ks = (int)(p % KS);
  const int n = 16 * j + (lane & 15), k0 = 32 * ks + 8 * (lane >> 4);
  bf16x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = W[(int64_t)(k0 + e) * N + n];
  *reinterpret_cast<bf16x8*>(Bt + i * 8) = v;
}

__global__ void ref_kernel(const bf16* A, const bf16* W, float* C, int M, int N, int K) {
  const int n = blockIdx.x * 256 + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(int64_t)m * K + k] * (float)W[(int64_t)k * N + n];
  C[(int64_t)m * N + n] = s;
}

// BM x BN tile, 4 waves splitting N (wave: BM x BN/4), k-tiles of 64 (two 32-deep k-steps);
// A rows through a 2-stage LDS ring filled from registers 2 k-tiles ahead; B from Bt in register
// batches of QB k-steps, double buffered.  Requires M % BM == 0, N % BN == 0, K % (32 QB) == 0,
// K / 64 >= 4.
template <int BM, int BN, int QB, int AD, int KT>
__global__ void __launch_bounds__(256) breg_kernel(const bf16* __restrict__ A, const bf16* __restrict__ Bt,
                                                   bf16* __restrict__ C, int M, int N, int K) {
  constexpr int FM = BM / 16, WN = BN / 4, FN = WN / 16;
  constexpr int TPB = QB / KT;            // k-tiles per B batch (a k-tile: KT 32-deep k-steps)
  constexpr int CPT = BM * KT * 4 / 256;  // 16-B A chunks per thread per k-tile
  constexpr int RB = KT * 64;             // LDS bytes per A row per stage
  static_assert(TPB % AD == 0 && AD % 2 == 0 && CPT >= 1, "shape");
  __shared__ __attribute__((aligned(16))) char sA[2][BM * RB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware tile order: XCD x (= blockIdx % 8) takes the x-th contiguous chunk of the M-major tile
  // list (its tiles share A row panels; every XCD reads all of B once into its L2)
  const int MT = M / BM, NT = N / BN, T = MT * NT;
  const int per = (T + 7) / 8;
  const int tile = (blockIdx.x % 8) * per + blockIdx.x / 8;
  if (tile >= T) return;
  const int mt = tile / NT, nt = tile % NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk = K / (32 * KT), nb = K / (32 * QB), KS = K / 32;

  const bf16* brow[FN];
#pragma unroll
  for (int f = 0; f < FN; ++f) brow[f] = Bt + ((int64_t)((n0 + w * WN) / 16 + f) * KS * 64 + lane) * 8;
  bf16x8 bq[2][QB][FN];
  auto loadB = [&](int b, bf16x8 (&dst)[QB][FN]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < QB; ++q)
#pragma unroll
      for (int f = 0; f < FN; ++f) dst[q][f] = *reinterpret_cast<const bf16x8*>(brow[f] + (int64_t)(b * QB + q) * 512);
  };
  u32x4 ar[AD][CPT];  // A(t) in ar[t % AD], loaded AD - 1 k-tiles before its LDS write
  auto loadA = [&](int kt, u32x4 (&r)[CPT]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int id = tid + 256 * c, row = id / (KT * 4), ch = id % (KT * 4);
      r[c] = *reinterpret_cast<const u32x4*>(A + (int64_t)(m0 + row) * K + kt * KT * 32 + ch * 8);
    }
  };
  auto writeA = [&](int st, const u32x4 (&r)[CPT]) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int id = tid + 256 * c, row = id / (KT * 4), ch = id % (KT * 4);
      *reinterpret_cast<u32x4*>(sA[st] + row * RB + ((ch ^ (row & 7)) * 16)) = r[c];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int f = 0; f < FN; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int i = 0; i < AD; ++i)
    if (i < nk) loadA(i, ar[i]);
  loadB(0, bq[0]);
  if (nb > 1) loadB(1, bq[1]);
  writeA(0, ar[0]);
  if (AD < nk) loadA(AD, ar[0]);

  // one B batch (QB k-steps = TPB k-tiles) from register buffer H (a compile-time index: a runtime
  // one sends the batches to scratch)
  auto batch = [&](int b, auto Hc) __attribute__((always_inline)) {
    constexpr int H = decltype(Hc)::value;
#pragma unroll
    for (int tt = 0; tt < TPB; ++tt) {
      const int t = b * TPB + tt;  // t % AD == tt % AD: TPB is a multiple of AD
      __syncthreads();             // A(t) visible in stage t & 1; stage (t + 1) & 1 free
      if (t + 1 < nk) {
        writeA((tt + 1) & 1, ar[(tt + 1) % AD]);
        if (t + 1 + AD < nk) loadA(t + 1 + AD, ar[(tt + 1) % AD]);
      }
      const char* st = sA[tt & 1];
#pragma unroll
      for (int ks = 0; ks < KT; ++ks) {
        bf16x8 af[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = 16 * i + (lane & 15), ch = 4 * ks + (lane >> 4);
          af[i] = *reinterpret_cast<const bf16x8*>(st + row * RB + ((ch ^ (row & 7)) * 16));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int f = 0; f < FN; ++f)
            acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[H][KT * tt + ks][f], af[i], acc[i][f], 0, 0, 0);
      }
    }
    if (b + 2 < nb) loadB(b + 2, bq[H]);
  };
  for (int bb = 0; bb < nb; bb += 2) {
    batch(bb, std::integral_constant<int, 0>{});
    if (bb + 1 < nb) batch(bb + 1, std::integral_constant<int, 1>{});
  }
  // lane holds C[m0 + 16 i + (lane & 15)][n0 + w WN + 16 f + 4 (lane >> 4) + 0..3]
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int f = 0; f < FN; ++f) {
      const int m = m0 + 16 * i + (lane & 15), n = n0 + w * WN + 16 * f + 4 * (lane >> 4);
      typedef __attribute__((ext_vector_type(4))) __bf16 b4;
      *reinterpret_cast<b4*>(C + (int64_t)m * N + n) =
          b4{(bf16)acc[i][f][0], (bf16)acc[i][f][1], (bf16)acc[i][f][2], (bf16)acc[i][f][3]};
    }
}

template <int BM, int BN, int QB, int AD, int KT = 2>
static void run(const char* name, int M, int N, int K, const bf16* A, const bf16* Bt, bf16* C, const float* Cref,
                hipStream_t s) {
  if (M % BM || N % BN || K % (32 * QB) || K / (32 * KT) < 4 || (BM * KT * 4) % 256) {
    std::printf("%-22s M=%d N=%d K=%d: shape not supported\n", name, M, N, K);
    return;
  }
  const int T = (M / BM) * (N / BN);
  const int grid = ((T + 7) / 8) * 8;
  auto launch = [&] { breg_kernel<BM, BN, QB, AD, KT><<<grid, 256, 0, s>>>(A, Bt, C, M, N, K); };
  launch();
  CK(hipStreamSynchronize(s));
  std::vector<uint16_t> hc((size_t)M * N);
  std::vector<float> hr((size_t)M * N);
  CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), Cref, hr.size() * 4, hipMemcpyDeviceToHost));
  double maxerr = 0, maxref = 0;
  for (size_t i = 0; i < hc.size(); ++i) {
    uint32_t u = (uint32_t)hc[i] << 16;
    float v;
    std::memcpy(&v, &u, 4);
    maxerr = std::fmax(maxerr, std::fabs(v - hr[i]));
    maxref = std::fmax(maxref, std::fabs(hr[i]));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 200;
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < R; ++r) launch();
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / R;
  std::printf("%-22s M=%5d N=%5d K=%5d  grid %4d  %7.2f us  %6.1f TF/s  max|err|/max|ref| %.2e\n", name, M, N, K, grid,
              us, 2.0 * M * N * K / us * 1e-6, maxerr / maxref);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // the C2 step's input-gradient shapes, then the C4 decode step's (beam 5: 1280 rows, greedy: 256)
  const int shapes[][3] = {{2304, 512, 2048}, {1216, 512, 2048}, {2304, 512, 1536}, {1216, 512, 1536},
                           {2304, 2048, 512}, {1216, 2048, 512}, {2304, 512, 512},  {1216, 512, 512},
                           {1280, 512, 512},  {1280, 1536, 512}, {1280, 2048, 512}, {1280, 512, 2048},
                           {256, 512, 512},   {256, 1536, 512},  {256, 2048, 512},  {256, 512, 2048}};
  for (auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    bf16 *A, *W, *Bt, *C;
    float* Cref;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&W, (size_t)K * N * 2));
    CK(hipMalloc(&Bt, (size_t)K * N * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&Cref, (size_t)M * N * 4));
    std::vector<uint16_t> h((size_t)std::max(M, N) * K);
    uint32_t st = 12345u + M + N + K;
    auto rnd = [&] {
      st = st * 1664525u + 1013904223u;
      float f = ((st >> 8) & 0xFFFF) / 65536.f - 0.5f;
      uint32_t u;
      std::memcpy(&u, &f, 4);
      return (uint16_t)(u >> 16);
    };
    for (size_t i = 0; i < (size_t)M * K; ++i) h[i] = rnd();
    CK(hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice));
    for (size_t i = 0; i < (size_t)K * N; ++i) h[i] = rnd();
    CK(hipMemcpy(W, h.data(), (size_t)K * N * 2, hipMemcpyHostToDevice));
    const int64_t thr = (int64_t)(N / 16) * (K / 32) * 64;
    tile_t_kernel<<<(unsigned)((thr + 255) / 256), 256, 0, s>>>(W, K, N, Bt);
    ref_kernel<<<dim3((N + 255) / 256, M), 256, 0, s>>>(A, W, Cref, M, N, K);
    CK(hipStreamSynchronize(s));
    run<64, 64, 4, 2>("breg 64x64 q4a2", M, N, K, A, Bt, C, Cref, s);
    run<32, 64, 8, 4>("breg 32x64 q8a4", M, N, K, A, Bt, C, Cref, s);
    run<64, 64, 8, 2, 4>("breg 64x64 q8a2 k128", M, N, K, A, Bt, C, Cref, s);
    run<32, 64, 8, 2, 4>("breg 32x64 q8a2 k128", M, N, K, A, Bt, C, Cref, s);
    run<32, 64, 16, 4, 4>("breg 32x64 q16a4 k128", M, N, K, A, Bt, C, Cref, s);
    run<64, 64, 16, 2, 8>("breg 64x64 q16a2 k256", M, N, K, A, Bt, C, Cref, s);
    run<32, 64, 16, 2, 8>("breg 32x64 q16a2 k256", M, N, K, A, Bt, C, Cref, s);
    CK(hipFree(A));
    CK(hipFree(W));
    CK(hipFree(Bt));
    CK(hipFree(C));
    CK(hipFree(Cref));
  }
  return 0;
}
