// capgen — fused self-attention front: Q/K/V projection + masked attention in one launch (qkv_attn.hip).
#pragma once
#include "attention.h"

namespace capgen {

// For every (image b, head h): [q_h | k_h | v_h] = X_b . Wqkv_h^T (cross: q_h only) (bf16, f32 accumulation, rounded
// to bf16 once) into qkv, then the attention of g on them into o.  g.q/k/v must describe qkv (they
// are what the backward reads); g.Lq == g.Lk == rows per image.
struct QkvAttn {
  AttnGeom g;
  const bf16* X = nullptr;  // row r of image b at X + (b * L + r) * ldx (cross: L = g.Lq)
  int64_t ldx = 0;
  const bf16* W = nullptr;  // Wqkv (cross: Wq) in the tiled layout of qkv_tile_weights
  int d = 0;
  bf16* qkv = nullptr;  // [B * L][ldqkv]: q | k | v (null: not stored)
  int64_t ldqkv = 0;
  bf16* o = nullptr;  // attention output, g.o_ld / g.o_bs
  // cross attention (DecoderBlock's second MHA, modules.py:195-197): only q = X . Wq^T is projected
  // (W = Wq [d][d], qkv = the q buffer); K / V come from g.k / g.v (the precomputed cross K/V)
  int cross = 0;
};
bool qkv_attn_ok(const QkvAttn& a);
// The fronts read their projection weights TILED: the 64 lanes' 16-B MFMA fragments of 16-row block j
// and 32-deep k-step ks (lane: row 16 j + (lane & 15), k = 32 ks + 8 (lane >> 4) .. + 7) are 1 KB
// contiguous at dst + (16 j + ks) * 512 elements (K = 512).  A fragment load is then one coalesced
// 1-KB piece (8 whole cache lines) instead of 16 rows x 64 B (measured: 19.3 -> 13.5 us per encoder
// front launch, tools/front_microbench.py).  src: R rows (R % 16 == 0) of [R][ld], nn.Linear layout.
void qkv_tile_weights(const bf16* src, int R, int64_t ld, bf16* dst, hipStream_t s);
void qkv_attn_fwd(const QkvAttn& a, hipStream_t s);

// The output side of an attention block's backward in ONE launch per (image, head): dO_h = dA_b .
// Wo[:, 64h .. 64h + 63] -- the input gradient of the output projection (modules.py:77 o_linear;
// dA = the gradient at the projection's output) read through the tiled Wo^T -- straight into the
// attention backward's dO image, then the MFMA attention backward of g (dq / dk / dv exactly as
// attention_bwd writes them).  bf16, head size 64, d = 512, Lq, Lk <= 64.
struct QkvBwd {
  AttnGeom g;                 // as for attention_bwd (g.o_ld / o_bs unused: dO never leaves the launch)
  const bf16* dA = nullptr;   // rows of image b at dA + (b * g.Lq + i) * ldda
  int64_t ldda = 0;
  const bf16* Wt = nullptr;   // Wo^T in the tiled layout (qkv_tile_weights_t)
  bf16* dq = nullptr;
  bf16* dk = nullptr;
  bf16* dv = nullptr;
};
bool qkv_bwd_ok(const QkvBwd& a);
void qkv_attn_bwd(const QkvBwd& a, hipStream_t s);
// qkv_tile_weights of W^T for a 512 x 512 nn.Linear weight W [out][in] (row stride ld): dst holds
// the [in][out] matrix tiled
void qkv_tile_weights_t(const bf16* src, int64_t ld, bf16* dst, hipStream_t s);

}  // namespace capgen
