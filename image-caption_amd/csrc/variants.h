// capgen — row-gather / row-reduce kernels of the reference's encoder/decoder variant flags.
// Off the measured C2 path (every flag defaults to False): plain grid-stride elementwise
// kernels over [rows, d] activations (act dtype, f32 arithmetic).
#pragma once
#include "capgen_common.h"
#include "gemm.h"

namespace capgen {

// ---- split_image_objects (model.py:258-292) ------------------------------------------------
// every region r = (b, n) becomes the 2-token sequence [Y[b*N], Y[r]]:
// X2[2r] = Y[b*N], X2[2r+1] = Y[r]; valid2 likewise (the pair's key-pad / non-pad mask)
void pair_gather(const void* Y, const uint8_t* valid, int B, int N, int d, void* X2, uint8_t* valid2, DType t,
                 hipStream_t s);
// out[r] = Z[2r+1] + Ep[r]   (the region token of the image block + its position embedding)
void pair_take_add(const void* Z, const void* Ep, int Me, int d, void* out, DType t, hipStream_t s);
// backward of pair_take_add: dZ[2r+1] = dA[r], dZ[2r] = 0
void pair_scatter(const void* dA, int Me, int d, void* dZ, DType t, hipStream_t s);
// backward of pair_gather: dY[r] = dX2[2r+1] + (n == 0 ? sum_n' dX2[2(b*N+n')] : 0)
void pair_reduce(const void* dX2, int B, int N, int d, void* dY, DType t, hipStream_t s);
// dst[i] += src[i], i < n
void add_inplace(void* dst, const void* src, int64_t n, DType t, hipStream_t s);

// ---- move_first_image_feature (model.py:451-457) ---------------------------------------------
// out[r] = D[r] + X[img(r) * N]; img(r) = bmod > 0 ? r % bmod : r / rows_per_img
void add_first_region(const void* D, const void* X, int R, int rows_per_img, int bmod, int N, int d, void* out,
                      DType t, hipStream_t s);
// backward into the encoder output: dX[b*N] += sum_{j < rows_per_img} dU[b*rows_per_img + j]
void first_region_grad(const void* dU, int B, int rows_per_img, int N, int d, void* dX, DType t, hipStream_t s);

}  // namespace capgen
