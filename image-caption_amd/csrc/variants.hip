// capgen — kernels of the reference's variant flags (variants.h).  One thread per element
// (f32 arithmetic, act-dtype storage); these shapes are small and off the measured path.
#include "variants.h"

namespace capgen {
namespace {

constexpr int TPB = 256;
inline int grid_for(int64_t n) { return (int)std::min<int64_t>((n + TPB - 1) / TPB, 65536); }

template <typename T>
__global__ void pair_gather_kernel(const T* __restrict__ Y, const uint8_t* __restrict__ valid, int N, int d,
                                   int64_t n, T* __restrict__ X2, uint8_t* __restrict__ valid2) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t r = i / d;
    const int c = (int)(i % d);
    const int64_t r0 = r / N * N;
    X2[2 * r * d + c] = Y[r0 * d + c];
    X2[(2 * r + 1) * d + c] = Y[i];
    if (c == 0) valid2[2 * r] = valid[r0], valid2[2 * r + 1] = valid[r];
  }
}

template <typename T>
__global__ void pair_take_add_kernel(const T* __restrict__ Z, const T* __restrict__ Ep, int d, int64_t n,
                                     T* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t r = i / d;
    const int c = (int)(i % d);
    out[i] = from_f<T>(to_f(Z[(2 * r + 1) * d + c]) + to_f(Ep[i]));
  }
}

template <typename T>
__global__ void pair_scatter_kernel(const T* __restrict__ dA, int d, int64_t n, T* __restrict__ dZ) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t r = i / d;
    const int c = (int)(i % d);
    dZ[2 * r * d + c] = from_f<T>(0.f);
    dZ[(2 * r + 1) * d + c] = dA[i];
  }
}

template <typename T>
__global__ void pair_reduce_kernel(const T* __restrict__ dX2, int N, int d, int64_t n, T* __restrict__ dY) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t r = i / d;
    const int c = (int)(i % d);
    float acc = to_f(dX2[(2 * r + 1) * d + c]);
    if (r % N == 0)
      for (int j = 0; j < N; ++j) acc += to_f(dX2[2 * (r + j) * d + c]);
    dY[i] = from_f<T>(acc);
  }
}

template <typename T>
__global__ void add_inplace_kernel(T* __restrict__ dst, const T* __restrict__ src, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
    dst[i] = from_f<T>(to_f(dst[i]) + to_f(src[i]));
}

template <typename T>
__global__ void add_first_region_kernel(const T* __restrict__ D, const T* __restrict__ X, int rows_per_img,
                                        int bmod, int N, int d, int64_t n, T* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t r = i / d;
    const int c = (int)(i % d);
    const int64_t img = bmod > 0 ? r % bmod : r / rows_per_img;
    out[i] = from_f<T>(to_f(D[i]) + to_f(X[img * N * d + c]));
  }
}

template <typename T>
__global__ void first_region_grad_kernel(const T* __restrict__ dU, int rows_per_img, int N, int d, int64_t n,
                                         T* __restrict__ dX) {
  for (int64_t i = blockIdx.x * (int64_t)TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t b = i / d;
    const int c = (int)(i % d);
    float acc = to_f(dX[b * N * d + c]);
    for (int j = 0; j < rows_per_img; ++j) acc += to_f(dU[(b * rows_per_img + j) * d + c]);
    dX[b * N * d + c] = from_f<T>(acc);
  }
}

}  // namespace

// launch KERNEL<bf16 | float> over n elements; `P(x)` casts an activation pointer to T*
#define CAPGEN_LAUNCH(t, n, KERNEL, ...)                                      \
  do {                                                                        \
    if ((n) > 0) {                                                            \
      if ((t) == DType::BF16) {                                               \
        typedef bf16 T;                                                       \
        KERNEL<T><<<grid_for(n), TPB, 0, s>>>(__VA_ARGS__);                   \
      } else {                                                                \
        typedef float T;                                                      \
        KERNEL<T><<<grid_for(n), TPB, 0, s>>>(__VA_ARGS__);                   \
      }                                                                       \
      CAPGEN_HIP(hipGetLastError());                                          \
    }                                                                         \
  } while (0)

void pair_gather(const void* Y, const uint8_t* valid, int B, int N, int d, void* X2, uint8_t* valid2, DType t,
                 hipStream_t s) {
  const int64_t n = (int64_t)B * N * d;
  CAPGEN_LAUNCH(t, n, pair_gather_kernel, (const T*)Y, valid, N, d, n, (T*)X2, valid2);
}

void pair_take_add(const void* Z, const void* Ep, int Me, int d, void* out, DType t, hipStream_t s) {
  const int64_t n = (int64_t)Me * d;
  CAPGEN_LAUNCH(t, n, pair_take_add_kernel, (const T*)Z, (const T*)Ep, d, n, (T*)out);
}

void pair_scatter(const void* dA, int Me, int d, void* dZ, DType t, hipStream_t s) {
  const int64_t n = (int64_t)Me * d;
  CAPGEN_LAUNCH(t, n, pair_scatter_kernel, (const T*)dA, d, n, (T*)dZ);
}

void pair_reduce(const void* dX2, int B, int N, int d, void* dY, DType t, hipStream_t s) {
  const int64_t n = (int64_t)B * N * d;
  CAPGEN_LAUNCH(t, n, pair_reduce_kernel, (const T*)dX2, N, d, n, (T*)dY);
}

void add_inplace(void* dst, const void* src, int64_t n, DType t, hipStream_t s) {
  CAPGEN_LAUNCH(t, n, add_inplace_kernel, (T*)dst, (const T*)src, n);
}

void add_first_region(const void* D, const void* X, int R, int rows_per_img, int bmod, int N, int d, void* out,
                      DType t, hipStream_t s) {
  const int64_t n = (int64_t)R * d;
  CAPGEN_LAUNCH(t, n, add_first_region_kernel, (const T*)D, (const T*)X, rows_per_img, bmod, N, d, n, (T*)out);
}

void first_region_grad(const void* dU, int B, int rows_per_img, int N, int d, void* dX, DType t, hipStream_t s) {
  const int64_t n = (int64_t)B * d;
  CAPGEN_LAUNCH(t, n, first_region_grad_kernel, (const T*)dU, rows_per_img, N, d, n, (T*)dX);
}

}  // namespace capgen
