// capgen — packed parameter arena layout (host only).
//
// The arena is one f32 allocation.  GEMM weights come first ("dense region",
// [0, n_dense)): they are fully overwritten by the weight-gradient GEMMs each step and
// mirrored into a bf16 shadow for the bf16 MFMA path.  Everything whose gradient is
// accumulated (word embedding table, LayerNorm gamma/beta, biases) follows, so one
// memset clears all accumulated gradients.  Weights that the hot path consumes
// together are adjacent: q/k/v of one attention block form one [3d, d] matrix (one
// fused QKV GEMM), the cross-attention k/v of ALL decoder blocks form one [Ld*2d, d]
// matrix (one GEMM over the encoder output), and the region-feature and position
// embeddings form one [d, Kp] matrix over the packed [feats | pos | 0] input.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/capgen.h"

namespace capgen {

struct EncLayerOff {
  int64_t Wqkv, Wo, W1, W2;            // dense
  int64_t ln1g, ln1b, b1, b2, ln2g, ln2b;
};
struct DecLayerOff {
  int64_t Wqkv, Wo_s, Wq_c, Wo_c, W1, W2;  // dense
  int64_t lsg, lsb, lcg, lcb, b1, b2, lfg, lfb;
};

struct Layout {
  // dims
  int V, maxlen, F, P, Kp, d, fe, Le, He, dwe, dd, fd, Ld, Hd;
  // dense region
  int64_t enc_emb_W = 0, Wel = 0, Wkv_all = 0, Wc = 0;
  std::vector<EncLayerOff> enc;
  std::vector<DecLayerOff> dec;
  // split_image_objects: encoder.image_encoder (dense weights inside the embedding bucket
  // [0, enc[0].Wqkv), small ones inside the encoder LN/bias region)
  bool has_img = false;
  EncLayerOff img{};
  // move_first_image_feature: the decoder's trailing FFN (dense weights inside the cross-K/V
  // bucket [Wkv_all, Wc), small ones inside the decoder LN/bias region)
  bool has_mf = false;
  int64_t mf_W1 = 0, mf_W2 = 0, mf_b1 = 0, mf_b2 = 0, mf_lng = 0, mf_lnb = 0;
  int64_t n_dense = 0;
  // accumulated region
  int64_t emb = 0, enc_lng = 0, enc_lnb = 0, dec_lng = 0, dec_lnb = 0, bc = 0;
  int64_t total = 0;
  std::vector<capgen_param_info> table;  // reference state_dict names
};

Layout make_layout(const capgen_config& c);
void validate_config(const capgen_config& c);

}  // namespace capgen
