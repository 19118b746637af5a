// capgen — shared device/host helpers for the gfx950 (MI355X, CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>
#include <string>

#include "capgen_host.h"

typedef __bf16 bf16;

#define CAPGEN_HIP(expr)                                                                  \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      throw capgen::Error(std::string(#expr) + ": " + hipGetErrorString(_e) + " at " +    \
                          __FILE__ + ":" + std::to_string(__LINE__));                     \
  } while (0)

namespace capgen {

// Debug build only (Knob::Skip bitmask): skip a kernel class to measure its marginal cost on the
// step's critical path.  1 LN fwd, 2 attention fwd, 4 LN bwd, 8 attention bwd, 16 GEMM f32-out
// (weight gradients + classifier), 32 Adam, 64 bf16 GEMMs, 128 LayerNorm-backward gamma/beta/bias sums.
inline int skip_mask() {
#ifdef CAPGEN_DEBUG
  return knob(Knob::Skip);
#else
  return 0;
#endif
}

// ---- diagnostic in-kernel timestamps (capgen_debug_stamps) --------------------------------
// A launch given a stamp slot (16 x u64) records the 100 MHz real-time counter: [0] when block 0
// starts, [1 + (block % 8)] the latest block end of that residue class (atomic max).  nullptr:
// nothing is recorded (one uniform branch per block).
__device__ __forceinline__ uint64_t rt_now() { return __builtin_amdgcn_s_memrealtime(); }
struct StampScope {
  uint64_t* p;
  __device__ __forceinline__ explicit StampScope(uint64_t* q) : p(q) {
    if (p && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) p[0] = rt_now();
  }
  // (the end: the last 16 blocks of the grid and every 32nd, one atomic each -- every block's atomic
  // cost the step ~0.4 ms; the last-dispatched blocks are the ones that finish last)
  __device__ __forceinline__ ~StampScope() {
    if (p && threadIdx.x == 0 && (blockIdx.x + 16 >= gridDim.x || (blockIdx.x & 31) == 0))
      atomicMax(reinterpret_cast<unsigned long long*>(p) + 1 + (blockIdx.x & 7), (unsigned long long)rt_now());
  }
};

// ---- write-through output stores ----------------------------------------------------------
// A plain store leaves its line dirty in the writing XCD's L2 and the end of the launch writes every
// such line back before the next dependent launch may start (MI355X_MICROARCH.md price list,
// 'boundary': + B / 6 TB/s for B dirty bytes).  An sc1 buffer store writes through at once
// (16-B sc1 store ~ plain store, same table), overlapped with the rest of the launch.  The base
// must be wave-uniform (a kernel argument); offsets are bytes (< 2 GB).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
}
typedef __attribute__((ext_vector_type(2))) unsigned int wt_u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned int wt_u32x4;
__device__ __forceinline__ void wt_store8(__amdgpu_buffer_rsrc_t r, uint32_t off, wt_u32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ void wt_store16(__amdgpu_buffer_rsrc_t r, uint32_t off, wt_u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16 /* sc1 */);
}
// N consecutive elements of T at byte offset `off` from the rsrc base (16-B pieces), write-through
template <typename T, int N>
__device__ __forceinline__ void store_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&in)[N]);
// write-through default: off (measured slower in the step, 4-round A/B 3.16-3.22 vs 3.04-3.17 ms: the
// end-of-launch write-back is not what the ~3 us kernel boundary is made of); callers may set wt = 1
inline int wt_default() { return 0; }

// ---- scalar conversions -------------------------------------------------------------
// (store_wt after the conversions below)
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// 16-byte vector of T: 4 floats or 8 bf16.
template <typename T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  typedef float4 type;
};
template <> struct Vec16<bf16> {
  static constexpr int N = 8;
  typedef uint4 type;
};

// Load/store `n` (=N per lane chunk) consecutive elements as f32.
template <typename T, int N>
__device__ __forceinline__ void load_f(const T* p, float (&out)[N]) {
  if constexpr (sizeof(T) * N == 16) {
    typedef typename Vec16<T>::type V;
    V v = *reinterpret_cast<const V*>(p);
    const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = to_f(e[i]);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = to_f(p[i]);
  }
}
template <typename T, int N>
__device__ __forceinline__ void store_f(T* p, const float (&in)[N]) {
  if constexpr (sizeof(T) * N == 16) {
    typedef typename Vec16<T>::type V;
    V v;
    T* e = reinterpret_cast<T*>(&v);
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = from_f<T>(in[i]);
    *reinterpret_cast<V*>(p) = v;
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = from_f<T>(in[i]);
  }
}

template <typename T, int N>
__device__ __forceinline__ void store_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&in)[N]) {
  constexpr int PER = 16 / sizeof(T);  // elements per 16-B piece
  static_assert(N % PER == 0, "store_wt: whole 16-B pieces");
#pragma unroll
  for (int p = 0; p < N / PER; ++p) {
    typedef typename Vec16<T>::type V;
    V v;
    T* e = reinterpret_cast<T*>(&v);
#pragma unroll
    for (int i = 0; i < PER; ++i) e[i] = from_f<T>(in[p * PER + i]);
    wt_store16(r, off + p * 16, __builtin_bit_cast(wt_u32x4, v));
  }
}

// A wave-uniform pointer the compiler must treat as an unknown SGPR value: a select between an
// optional input and a device dummy stays a select (hipcc otherwise turns it back into a branch
// around the load, and waits for the load at the branch's join -- one memory round trip each).
template <typename P>
__device__ __forceinline__ P* opaque(P* p) {
  uint64_t v = reinterpret_cast<uint64_t>(p);
  asm volatile("" : "+s"(v));
  return reinterpret_cast<P*>(v);
}

// ---- wave64 reductions ----------------------------------------------------------------
// Lane exchanges inside a 16-lane row are DPP moves (a VALU operand modifier, no LDS crossbar):
// quad_perm swaps lanes ^1 and ^2, row_half_mirror pairs lane i with 7 - i (the other quad of the
// same 8), row_ror:8 is exactly lane ^ 8.  Across rows (^16, ^32) they go through ds_bpermute.
// For a commutative reduction of a value held by every lane, a mirror pairs a lane with one of
// the complementary half as well as an xor does (every lane ends with the group total).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // lane i <-> 7 - i within 8
constexpr int kDppRor8 = 0x128;        // lane i <-> i ^ 8 within 16
// lane ^ O (or, for O = 4, the half-mirror partner): DPP inside a row, ds_bpermute across rows
template <int O>
__device__ __forceinline__ int lane_xchg(int v) {
  if constexpr (O == 1) return __builtin_amdgcn_mov_dpp(v, kDppXor1, 0xf, 0xf, false);
  else if constexpr (O == 2) return __builtin_amdgcn_mov_dpp(v, kDppXor2, 0xf, 0xf, false);
  else if constexpr (O == 4) return __builtin_amdgcn_mov_dpp(v, kDppHalfMirror, 0xf, 0xf, false);
  else if constexpr (O == 8) return __builtin_amdgcn_mov_dpp(v, kDppRor8, 0xf, 0xf, false);
  else return __shfl_xor(v, O, 64);
}
template <int O>
__device__ __forceinline__ float lane_xchg(float v) {
  return __int_as_float(lane_xchg<O>(__float_as_int(v)));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<kDppXor1>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  v += dpp_f<kDppRor8>(v);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<kDppXor1>(v));
  v = fmaxf(v, dpp_f<kDppXor2>(v));
  v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_f<kDppRor8>(v));
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}

// ---- counter-based dropout RNG --------------------------------------------------------
// keep(seed, site, idx): a 32-bit avalanche hash (lowbias32: 2 multiplies, 3 xor-shifts) of the
// element index xored with a per-(step seed, site) key.  The key is the same hash of the seed and
// site, loop-invariant in every kernel (hoisted), so a mask element costs ~9 32-bit VALU operations
// (the splitmix64 finaliser of rounds 1-4 took ~3x that in 64-bit multiplies -- it is evaluated per
// attention probability and per LayerNorm element, in the forward and again in the backward).
// Masks are regenerated bit-identically in the backward pass, so nothing is stored.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_key(uint64_t seed, uint32_t site) {
  return lowbias32((uint32_t)seed ^ lowbias32((uint32_t)(seed >> 32) + 0x9E3779B9u * (site + 1u)));
}
__device__ __forceinline__ uint32_t mix32(uint64_t seed, uint32_t site, uint32_t idx) {
  return lowbias32(idx ^ drop_key(seed, site));
}
// true = keep.  p in [0,1).  threshold = p * 2^32.
__device__ __forceinline__ bool drop_keep(uint64_t seed, uint32_t site, uint32_t idx, uint32_t thresh) {
  return mix32(seed, site, idx) >= thresh;
}
inline uint32_t drop_threshold(float p) {
  double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// Dropout descriptor passed by value to kernels.  `seed_ptr` points at the device-side
// step seed so a captured hipGraph replays with a fresh mask each step.
struct Drop {
  const uint64_t* seed_ptr;  // null => dropout off
  uint32_t site;
  uint32_t thresh;
  float scale;  // 1/(1-p)
};

// one torch.optim.Adam element update (torch 2.x single-tensor path, no weight decay):
// neg_step = -lr / (1 - b1^t), bc2s = sqrt(1 - b2^t); b1c = 1 - b1, b2c = 1 - b2
__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float b1c, float b2, float b2c,
                                         float eps, float neg_step, float bc2s) {
  m = m + b1c * (g - m);                      // exp_avg.lerp_(grad, 1 - beta1)
  v = v * b2 + b2c * (g * g);                 // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  const float denom = sqrtf(v) / bc2s + eps;  // (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
  p = p + (neg_step * m) / denom;             // param.addcdiv_(exp_avg, denom, value=-step_size)
}

// Row mask applied to a LayerNorm output / its gradient: row m is zeroed when
// ids[m] == pad (decoder non_pad_mask, model.py:483-486) or valid[m] == 0 (encoder
// non_pad_mask with encode_mask, model.py:356-359).
struct RowMask {
  const int32_t* ids = nullptr;
  int64_t ids_ld = 1;  // ids of row m at ids[m * ids_ld]
  int pad_idx = 0;
  const uint8_t* valid = nullptr;
};

__device__ __forceinline__ bool row_kept(const RowMask& rm, int m) {
  if (rm.ids && rm.ids[(int64_t)m * rm.ids_ld] == rm.pad_idx) return false;
  if (rm.valid && !rm.valid[m]) return false;
  return true;
}

}  // namespace capgen
