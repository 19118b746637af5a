// capgen — fused self-attention front: Q/K/V projection + masked attention in one launch (qkv_attn.hip).
#pragma once
#include "attention.h"

namespace capgen {

// For every (image b, head h): [q_h | k_h | v_h] = X_b . Wqkv_h^T (cross: q_h only) (bf16, f32 accumulation, rounded
// to bf16 once) into qkv, then the attention of g on them into o.  g.q/k/v must describe qkv (they
// are what the backward reads); g.Lq == g.Lk == rows per image.
struct QkvAttn {
  AttnGeom g;
  const bf16* X = nullptr;  // row r of image b at X + b * x_bs + r * ldx
  int64_t ldx = 0;
  int64_t x_bs = -1;        // -1: L * ldx (images' rows contiguous); beam decode: the rows of image b
                            // are r = j * B + b, so ldx = B * d and x_bs = d
  const bf16* W = nullptr;  // Wqkv [3d][ldw] (nn.Linear layout)
  int64_t ldw = 0;
  int d = 0;
  bf16* qkv = nullptr;  // [B * L][ldqkv]: q | k | v (null: not stored, decode)
  int64_t ldqkv = 0;
  bf16* o = nullptr;  // attention output, g.o_ld / g.o_bs
  // cross attention (DecoderBlock's second MHA, modules.py:195-197): only q = X . Wq^T is projected
  // (W = Wq [d][d], qkv = the q buffer); K / V come from g.k / g.v (the precomputed cross K/V)
  int cross = 0;
};
bool qkv_attn_ok(const QkvAttn& a);
void qkv_attn_fwd(const QkvAttn& a, hipStream_t s);

// One KV-cached decode step of a decoder block's self attention (model.py:101-200 restated with a
// cache) for kb rows per image (beam rows r = j * B + image): [q | k | v] = x_r . Wqkv^T, k / v stored
// into the row's cache at position t, then row r attends over positions 0..t -- position p < t from
// cache row kv_row[r][p] (the beam it descends from; kv_row null: r itself), position t from the
// fresh projection -- with the key mask ids[r][p] == pad (causal by construction).  One workgroup per
// (image, head); the q projection never leaves the workgroup.
struct QkvDecode {
  int B = 0, H = 0, kb = 0, t = 0, d = 0;
  int prio = 0;
  const bf16* X = nullptr;  // row r at X + r * d
  const bf16* W = nullptr;  // Wqkv [3d][d]
  bf16* cache = nullptr;    // row r, position p: K at cache + r * c_ld + p * 2d, V at + d
  int64_t c_ld = 0;
  const int32_t* kv_row = nullptr;  // [rows][kv_row_ld]
  int64_t kv_row_ld = 0;
  const int32_t* ids = nullptr;  // [rows][ids_ld]
  int64_t ids_ld = 0;
  int pad_idx = 0;
  float temperature = 8.f;
  bf16* o = nullptr;  // row r at o + r * d
  uint64_t* stamp = nullptr;
};
bool qkv_decode_ok(const QkvDecode& a);
void qkv_decode_self(const QkvDecode& a, hipStream_t s);

}  // namespace capgen
