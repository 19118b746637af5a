// capgen — GEMM front end + the f32 parity-mode kernel (bf16 path: gemm_bf16.hip).
//
//   C[m][n] = epi( alpha * sum_k opA(m,k) * opB(k,n) )
//   opA(m,k) = TA ? A[k*lda + m] : A[m*lda + k]
//   opB(k,n) = TB ? B[k*ldb + n] : B[n*ldb + k]        (TB=0 is nn.Linear's W[N][K])
//   epi: (+ bias[n]) -> (* (aux[m][n] > 0)) -> relu -> (+ C_old if beta)
//
// Forward projections are NT (X . W^T), input gradients NN (dY . W), weight gradients
// TN (dY^T . X).  bf16 operands use v_mfma_f32_16x16x32_bf16; the fp32 parity mode
// uses v_mfma_f32_16x16x4_f32 (an exact f32 fma chain).  Accumulation is always f32.
//
// Tiling: 256 threads = 4 wave64s in a 2x2 grid over a BMxBN tile, BK = 32, two LDS
// buffers with register-staged global loads (issue next tile's loads before the MFMAs of
// the current tile, write them to the other LDS buffer after).  Transposed operands are
// transposed on the LDS write so every MFMA fragment is one 16-B ds_read (bf16).
#include <chrono>
#include <cstdio>
#include <vector>
#include "gemm.h"
#include "hazard.h"
#include "ops.h"

namespace capgen {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <typename T> struct GemmTraits;
template <> struct GemmTraits<float> {
  static constexpr int VEC = 4;  // elements per 16-B global load
  static constexpr int PAD = 4;
};
template <> struct GemmTraits<bf16> {
  static constexpr int VEC = 8;
  static constexpr int PAD = 8;
};

constexpr int BK = 32;
constexpr int NTHREADS = 256;

template <typename T, bool TRANS, int ROWS>
struct TileLoader {
  // Stage a ROWS x BK tile (rows = M or N index, cols = k) into registers, then LDS [ROWS][LDK].
  static constexpr int VEC = GemmTraits<T>::VEC;
  static constexpr int LDK = BK + GemmTraits<T>::PAD;
  static constexpr int NV = ROWS * BK / VEC / NTHREADS;  // vectors per thread
  static_assert(NV >= 1, "tile too small");
  typedef typename Vec16<T>::type V;
  V reg[NV];

  __device__ __forceinline__ void load(const T* __restrict__ src, int64_t ld, int r0, int R, int k0,
                                       int K, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int v = tid + i * NTHREADS;
      int r, k;
      bool ok;
      const T* p;
      if constexpr (!TRANS) {
        r = v / (BK / VEC);
        k = (v % (BK / VEC)) * VEC;
        ok = (r0 + r < R) && (k0 + k < K);
        p = src + (int64_t)(r0 + r) * ld + (k0 + k);
      } else {
        k = v / (ROWS / VEC);
        r = (v % (ROWS / VEC)) * VEC;
        ok = (k0 + k < K) && (r0 + r < R);
        p = src + (int64_t)(k0 + k) * ld + (r0 + r);
      }
      if (ok) {
        reg[i] = *reinterpret_cast<const V*>(p);
      } else {
        reg[i] = V{};
      }
    }
  }
  __device__ __forceinline__ void store(T* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int v = tid + i * NTHREADS;
      if constexpr (!TRANS) {
        int r = v / (BK / VEC);
        int k = (v % (BK / VEC)) * VEC;
        *reinterpret_cast<V*>(lds + r * LDK + k) = reg[i];
      } else {
        int k = v / (ROWS / VEC);
        int r = (v % (ROWS / VEC)) * VEC;
        const T* e = reinterpret_cast<const T*>(&reg[i]);
#pragma unroll
        for (int j = 0; j < VEC; ++j) lds[(r + j) * LDK + k] = e[j];
      }
    }
  }
};

template <typename T, typename TO, bool TA, bool TB, int BM, int BN>
__global__ void __launch_bounds__(NTHREADS) gemm_kernel(GemmArgs g) {
  constexpr int LDK = BK + GemmTraits<T>::PAD;
  constexpr int FM = BM / 32, FN = BN / 32;  // 16x16 fragments per wave
  __shared__ __attribute__((aligned(16))) T As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * LDK];

  const T* __restrict__ A = reinterpret_cast<const T*>(g.A);
  const T* __restrict__ B = reinterpret_cast<const T*>(g.B);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  TileLoader<T, TA, BM> la;
  TileLoader<T, TB, BN> lb;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + BK - 1) / BK;
  la.load(A, g.lda, m0, g.M, 0, g.K, tid);
  lb.load(B, g.ldb, n0, g.N, 0, g.K, tid);
  la.store(As[0], tid);
  lb.store(Bs[0], tid);
  __syncthreads();

  // f32 operands: three-level blocked accumulation -- each 64-deep K panel is summed in `acc` (a
  // 64-fma chain), four panels in `mid`, and the 256-deep sums in `tot`: ~64 + 4 + K/256 chained
  // roundings per output instead of K (a single chain at K = 2304 was ~5x further from the float64
  // result than the reference's CPU arithmetic on the cancelling random-init weight gradients; one
  // 256-deep level left encoder block 0's FFN-up gradient at ~3x the CPU's error, round 4)
  constexpr int KP1 = 64 / BK, KP2 = 4;
  f32x4 mid[FM][FN], tot[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) mid[i][j] = tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if constexpr (sizeof(T) == 4) {
      if (kt > 0 && kt % KP1 == 0) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) mid[i][j] += acc[i][j], acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (kt % (KP1 * KP2) == 0) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) tot[i][j] += mid[i][j], mid[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
    if (kt + 1 < nk) {
      la.load(A, g.lda, m0, g.M, (kt + 1) * BK, g.K, tid);
      lb.load(B, g.ldb, n0, g.N, (kt + 1) * BK, g.K, tid);
    }
    const T* as = As[cur] + (wm * (BM / 2) + fr) * LDK;
    const T* bs = Bs[cur] + (wn * (BN / 2) + fr) * LDK;
    if constexpr (sizeof(T) == 2) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(as + i * 16 * LDK + fq * 8);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(bs + j * 16 * LDK + fq * 8);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        float af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = to_f(as[i * 16 * LDK + ks * 4 + fq]);
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = to_f(bs[j * 16 * LDK + ks * 4 + fq]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) {
      la.store(As[cur ^ 1], tid);
      lb.store(Bs[cur ^ 1], tid);
    }
    __syncthreads();
  }

  if constexpr (sizeof(T) == 4) {
    if (nk > KP1) {  // (K <= 64: the chain alone)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = tot[i][j] + (mid[i][j] + acc[i][j]);
    }
  }
  // ---- epilogue ----
  const float alpha = g.alpha_ptr ? g.alpha * *g.alpha_ptr : g.alpha;
  TO* __restrict__ C = reinterpret_cast<TO*>(g.C);
  const T* __restrict__ aux = reinterpret_cast<const T*>(g.aux);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + fr;
      if (n >= g.N) continue;
      const float bn = g.bias ? g.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + i * 16 + fq * 4 + r;
        if (m >= g.M) continue;
        float v = alpha * acc[i][j][r] + bn;
        if (aux && !(to_f(aux[(int64_t)m * g.ldaux + n]) > 0.f)) v = 0.f;
        if (g.relu) v = fmaxf(v, 0.f);
        TO* cp = C + (int64_t)m * g.ldc + n;
        if (g.beta) v += to_f(*cp);
        *cp = from_f<TO>(v);
      }
    }
  }
}

template <typename T, typename TO, bool TA, bool TB>
static void launch_tiles(const GemmArgs& g, hipStream_t s) {
  // Pick the largest tile that still gives >= ~1 block per CU (256 CUs).
  auto blocks = [&](int bm, int bn) { return (long)((g.M + bm - 1) / bm) * ((g.N + bn - 1) / bn); };
  if (blocks(128, 128) >= 240) {
    dim3 grid((g.N + 127) / 128, (g.M + 127) / 128);
    gemm_kernel<T, TO, TA, TB, 128, 128><<<grid, NTHREADS, 0, s>>>(g);
  } else if (blocks(128, 64) >= 240) {
    dim3 grid((g.N + 63) / 64, (g.M + 127) / 128);
    gemm_kernel<T, TO, TA, TB, 128, 64><<<grid, NTHREADS, 0, s>>>(g);
  } else {
    dim3 grid((g.N + 63) / 64, (g.M + 63) / 64);
    gemm_kernel<T, TO, TA, TB, 64, 64><<<grid, NTHREADS, 0, s>>>(g);
  }
}

template <typename T, typename TO>
static void launch_layout(const GemmArgs& g, bool ta, bool tb, hipStream_t s) {
  if (!ta && !tb) launch_tiles<T, TO, false, false>(g, s);
  else if (!ta && tb) launch_tiles<T, TO, false, true>(g, s);
  else if (ta && !tb) launch_tiles<T, TO, true, false>(g, s);
  else launch_tiles<T, TO, true, true>(g, s);
}

// the device bytes one GEMM touches (hazard checker, hazard.h; also used by gemm_grouped)
void gemm_hz_regions(const GemmArgs& g, DType in, DType out, bool ta, bool tb, std::vector<hz::Rgn>& v) {
  using namespace hz;
  const int64_t ei = dsize(in), eo = dsize(out);
  const int ncol = g.C2 ? g.nsplit : g.N;
  v.push_back(g.a_ids ? blk(g.A, g.a_table_rows, g.K * ei, g.lda * ei, RD)
                      : ta ? blk(g.A, g.K, g.M * ei, g.lda * ei, RD) : blk(g.A, g.M, g.K * ei, g.lda * ei, RD));
  v.push_back(blk(g.a_ids, g.a_ids ? g.M : 0, 4, g.a_ids_ld * 4, RD));
  v.push_back(tb ? blk(g.B, g.K, g.N * ei, g.ldb * ei, RD) : blk(g.B, g.N, g.K * ei, g.ldb * ei, RD));
  v.push_back(blk(g.C, g.M, ncol * eo, g.ldc * eo, WR));
  if (g.beta) v.push_back(blk(g.C, g.M, ncol * eo, g.ldc * eo, RD));
  if (g.C2) v.push_back(blk(g.C2, g.M, (int64_t)(g.N - g.nsplit) * eo, g.ldc2 * eo, WR));
  v.push_back(blk(g.aux, g.M, g.N * ei, g.ldaux * ei, RD));
  v.push_back(rd(g.bt, (int64_t)g.N * g.K * 2));
  v.push_back(rd(g.bias, g.N * 4));
  v.push_back(rd(g.alpha_ptr, 4));
  v.push_back(blk(g.colsum, g.colsum_stripes, g.N * 4, g.colsum_stride * 4, ACC));
  v.push_back(blk(g.ce_stats, g.M, (int64_t)((g.N + 15) / 16) * 8, g.ce_ld * 8, WR));
  v.push_back(blk(g.dec_stats, g.M, (int64_t)((g.N + 15) / 16) * 8, g.dec_ld * 8, WR));
  v.push_back(rd(g.ce_tgt, (int64_t)g.M * 4));
  v.push_back(wr(g.ce_tlogit, (int64_t)g.M * 4));
  v.push_back(rd(g.ln_gamma, g.K * 4));
  v.push_back(rd(g.ln_beta, g.K * 4));
  v.push_back(blk(g.ln_ids, g.ln_ids ? g.M : 0, 4, g.ln_ids_ld * 4, RD));
  v.push_back(wr(g.ln_y, (int64_t)g.M * g.K * 2));
  v.push_back(rd(g.ln_res, (int64_t)g.M * g.K * 2));
}

static void gemm_impl(const GemmArgs& g, DType in, DType out, bool ta, bool tb, hipStream_t s);
// debug build, Knob::HostTiming: average host time of a gemm() call, printed every 2000 calls
void gemm(const GemmArgs& g, DType in, DType out, bool ta, bool tb, hipStream_t s) {
  if (!knob(Knob::HostTiming)) return gemm_impl(g, in, out, ta, tb, s);
  static double tot = 0;
  static long n = 0;
  const auto t0 = std::chrono::steady_clock::now();
  gemm_impl(g, in, out, ta, tb, s);
  tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  if (++n % 2000 == 0) {
    std::fprintf(stderr, "[capgen host] gemm() call: %.2f us average over 2000\n", tot / 2000);
    tot = 0;
  }
}
static void gemm_impl(const GemmArgs& g, DType in, DType out, bool ta, bool tb, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return;
  if ((skip_mask() & 16) && out == DType::F32) return;
  if ((skip_mask() & 64) && out == DType::BF16) return;
  const int vec = in == DType::F32 ? 4 : 8;
  // the contiguous dimension of each operand is read in 16-B vectors
  require((ta ? g.M : g.K) % vec == 0 && g.lda % vec == 0, "gemm: A contiguous dim/ld not a multiple of 16 B");
  require((tb ? g.N : g.K) % vec == 0 && g.ldb % vec == 0, "gemm: B contiguous dim/ld not a multiple of 16 B");
  require(((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0, "gemm: operands must be 16-B aligned");
  require(g.K > 0, "gemm: K must be positive");
  require(!g.colsum || !g.beta, "gemm: colsum requires beta == 0");
  require(!g.bt || (in == DType::BF16 && !ta), "gemm: a tiled B (bt) needs the bf16 path with A stored [M][K]");
  require(!g.dec_stats || in == DType::BF16, "gemm: dec_stats is a bf16-path epilogue output");
  require(!g.a_ids || (in == DType::BF16 && !ta && !tb && g.bt && gemm_breg_ok(g) && g.a_table_rows > 0),
          "gemm: gathered A rows (a_ids) need the register-B path");
  require(!g.ln_gamma || (in == DType::BF16 && !ta && !tb && g.bt && gemm_breg_ok(g)),
          "gemm: a folded LayerNorm (ln_gamma) needs the register-B path (bf16, bt, K = 512)");
  require(!g.C2 || (in == DType::BF16 && g.nsplit % 4 == 0 && !g.beta && !g.colsum),
          "gemm: a split output (C2) needs the bf16 path, nsplit % 4 == 0, no beta / colsum");
  if (hz::active()) {
    std::vector<hz::Rgn> v;
    gemm_hz_regions(g, in, out, ta, tb, v);
    hz::op(s, ta ? "gemm TN (dW)" : tb ? "gemm NN (dX)" : "gemm NT (fwd)", v.data(), v.size());
  }
  if (in == DType::F32) {
    if (out == DType::F32) launch_layout<float, float>(g, ta, tb, s);
    else launch_layout<float, bf16>(g, ta, tb, s);
    if (g.colsum) column_sum(g.C, g.M, g.N, g.ldc, 1.f, nullptr, g.colsum, out, s, g.colsum_stripes, g.colsum_stride);
  } else {
    gemm_bf16(g, out, ta, tb, s);
  }
  CAPGEN_HIP(hipGetLastError());
}

}  // namespace capgen
