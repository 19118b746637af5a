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

}  // namespace capgen
