// capgen — packed parameter arena layout and the reference-name table (host only).
#include "layout.h"

#include <cstring>

#include "capgen_host.h"

namespace capgen {

void validate_config(const capgen_config& c) {
  require(c.num_vocab > 0 && c.num_vocab % 8 == 0, "config: num_vocab must be a positive multiple of 8");
  require(c.max_length >= 2 && c.max_length - 1 <= 64, "config: max_length must be in [2, 65]");
  require(c.dim_features > 0 && c.dim_features % 8 == 0, "config: dim_features must be a multiple of 8");
  require(c.dim_positions > 0, "config: dim_positions must be positive");
  require(!c.split_position || c.dim_positions > 4, "config: split_position needs dim_positions > 4");
  // model.py:258-292 applies position_embedding to the full position row, which a split
  // Linear(4, d) cannot take: the reference itself fails on this combination
  require(!(c.split_position && c.split_image_objects), "config: split_position and split_image_objects exclude "
          "each other");
  require(!c.split_image_objects || c.enc_blocks >= 1, "config: split_image_objects needs >= 1 encoder block");
  require(c.enc_d == c.dec_d, "config: encoder and decoder widths must match");
  require(c.enc_d % 64 == 0 && c.enc_d <= 1024 && ((c.enc_d / 64) & (c.enc_d / 64 - 1)) == 0,
          "config: model width must be 64 * {1,2,4,8,16}");
  require(c.enc_heads > 0 && c.enc_d % c.enc_heads == 0 && (c.enc_d / c.enc_heads) % 8 == 0 &&
              c.enc_d / c.enc_heads <= 128,
          "config: encoder head size must be a multiple of 8 and <= 128");
  require(c.dec_heads > 0 && c.dec_d % c.dec_heads == 0 && (c.dec_d / c.dec_heads) % 8 == 0 &&
              c.dec_d / c.dec_heads <= 128,
          "config: decoder head size must be a multiple of 8 and <= 128");
  require(c.enc_ff % 8 == 0 && c.dec_ff % 8 == 0, "config: FFN widths must be multiples of 8");
  require(c.dim_word_embedding % 8 == 0, "config: dim_word_embedding must be a multiple of 8");
  require(c.enc_blocks >= 0 && c.dec_blocks >= 1, "config: need >= 1 decoder block");
  require(c.dtype == CAPGEN_F32 || c.dtype == CAPGEN_BF16, "config: dtype must be CAPGEN_F32 or CAPGEN_BF16");
  require(c.dropout >= 0.f && c.dropout < 1.f && c.attention_dropout >= 0.f && c.attention_dropout < 1.f,
          "config: dropout must be in [0, 1)");
}

namespace {
struct Builder {
  Layout& L;
  int64_t cur = 0;
  int64_t take(int64_t n) {
    int64_t off = (cur + 63) / 64 * 64;  // 256-B aligned tensors
    cur = off + n;
    return off;
  }
  void name(const std::string& n, int ndim, int64_t rows, int64_t cols, int64_t off, int64_t stride) {
    capgen_param_info p;
    std::memset(&p, 0, sizeof(p));
    require(n.size() < sizeof(p.name), "layout: parameter name too long");
    std::memcpy(p.name, n.c_str(), n.size());
    p.ndim = ndim;
    p.rows = rows;
    p.cols = cols;
    p.offset = off;
    p.row_stride = stride;
    L.table.push_back(p);
  }
  void mat(const std::string& n, int64_t rows, int64_t cols, int64_t off) { name(n, 2, rows, cols, off, cols); }
  void vec(const std::string& n, int64_t len, int64_t off) { name(n, 1, 1, len, off, len); }
};
}  // namespace

Layout make_layout(const capgen_config& c) {
  validate_config(c);
  Layout L;
  L.V = c.num_vocab;
  L.maxlen = c.max_length;
  L.F = c.dim_features;
  L.P = c.dim_positions;
  L.Kp = (L.F + L.P + 63) / 64 * 64;
  L.d = c.enc_d;
  L.fe = c.enc_ff;
  L.Le = c.enc_blocks;
  L.He = c.enc_heads;
  L.dwe = c.dim_word_embedding;
  L.dd = c.dec_d;
  L.fd = c.dec_ff;
  L.Ld = c.dec_blocks;
  L.Hd = c.dec_heads;
  const int64_t d = L.d, dd = L.dd;
  Builder b{L};

  // ---- dense region (GEMM weights) ----
  L.enc_emb_W = b.take(d * L.Kp);
  L.has_img = c.split_image_objects != 0;
  if (L.has_img) {
    L.img.Wqkv = b.take(3 * d * d);
    L.img.Wo = b.take(d * d);
    L.img.W1 = b.take((int64_t)L.fe * d);
    L.img.W2 = b.take(d * L.fe);
  }
  L.enc.resize(L.Le);
  for (auto& e : L.enc) {
    e.Wqkv = b.take(3 * d * d);
    e.Wo = b.take(d * d);
    e.W1 = b.take((int64_t)L.fe * d);
    e.W2 = b.take(d * L.fe);
  }
  L.Wel = b.take(dd * L.dwe);
  L.dec.resize(L.Ld);
  for (auto& e : L.dec) {
    e.Wqkv = b.take(3 * dd * dd);
    e.Wo_s = b.take(dd * dd);
    e.Wq_c = b.take(dd * dd);
    e.Wo_c = b.take(dd * dd);
    e.W1 = b.take((int64_t)L.fd * dd);
    e.W2 = b.take(dd * L.fd);
  }
  L.Wkv_all = b.take((int64_t)L.Ld * 2 * dd * d);
  L.has_mf = c.move_first_image_feature != 0;
  if (L.has_mf) {
    L.mf_W1 = b.take((int64_t)L.fd * dd);
    L.mf_W2 = b.take(dd * L.fd);
  }
  L.Wc = b.take((int64_t)L.V * dd);
  L.n_dense = (b.cur + 63) / 64 * 64;
  b.cur = L.n_dense;

  // ---- accumulated region ----
  L.emb = b.take((int64_t)L.V * L.dwe);
  L.enc_lng = b.take(d);
  L.enc_lnb = b.take(d);
  if (L.has_img) {
    auto& e = L.img;
    e.ln1g = b.take(d);
    e.ln1b = b.take(d);
    e.b1 = b.take(L.fe);
    e.b2 = b.take(d);
    e.ln2g = b.take(d);
    e.ln2b = b.take(d);
  }
  for (auto& e : L.enc) {
    e.ln1g = b.take(d);
    e.ln1b = b.take(d);
    e.b1 = b.take(L.fe);
    e.b2 = b.take(d);
    e.ln2g = b.take(d);
    e.ln2b = b.take(d);
  }
  L.dec_lng = b.take(dd);
  L.dec_lnb = b.take(dd);
  if (L.has_mf) {
    L.mf_b1 = b.take(L.fd);
    L.mf_b2 = b.take(dd);
    L.mf_lng = b.take(dd);
    L.mf_lnb = b.take(dd);
  }
  for (auto& e : L.dec) {
    e.lsg = b.take(dd);
    e.lsb = b.take(dd);
    e.lcg = b.take(dd);
    e.lcb = b.take(dd);
    e.b1 = b.take(L.fd);
    e.b2 = b.take(dd);
    e.lfg = b.take(dd);
    e.lfb = b.take(dd);
  }
  L.bc = b.take(L.V);
  L.total = (b.cur + 63) / 64 * 64;

  // ---- reference names, registration order (model.py:44-69; modules.py:42-62, 100-107) ----
  // split_position (model.py:231-233, 297-303): feats.W_f^T + pos[:, :4].W_p^T + pos[:, 4:].W_o^T is
  // the one packed product over [feats | pos]; only the names of the position columns change
  // (object_embedding registered first, model.py:231-233)
  if (c.split_position) {
    b.name("encoder.object_embedding.weight", 2, d, L.P - 4, L.enc_emb_W + L.F + 4, L.Kp);
    b.name("encoder.position_embedding.weight", 2, d, 4, L.enc_emb_W + L.F, L.Kp);
  } else {
    b.name("encoder.position_embedding.weight", 2, d, L.P, L.enc_emb_W + L.F, L.Kp);
  }
  auto enc_block = [&](const EncLayerOff& e, const std::string& p) {
    const std::string m = p + "multihead_attention.";
    b.mat(m + "q_linear.weight", d, d, e.Wqkv);
    b.mat(m + "k_linear.weight", d, d, e.Wqkv + d * d);
    b.mat(m + "v_linear.weight", d, d, e.Wqkv + 2 * d * d);
    b.vec(m + "layer_norm.weight", d, e.ln1g);
    b.vec(m + "layer_norm.bias", d, e.ln1b);
    b.mat(m + "joint_linear.weight", d, d, e.Wo);
    const std::string f = p + "feed_forward.";
    b.mat(f + "position_wise_1.weight", L.fe, d, e.W1);
    b.vec(f + "position_wise_1.bias", L.fe, e.b1);
    b.mat(f + "position_wise_2.weight", d, L.fe, e.W2);
    b.vec(f + "position_wise_2.bias", d, e.b2);
    b.vec(f + "layer_norm.weight", d, e.ln2g);
    b.vec(f + "layer_norm.bias", d, e.ln2b);
  };
  if (L.has_img) enc_block(L.img, "encoder.image_encoder.");  // model.py:237-244: after position_embedding
  b.name("encoder.feature_embedding.weight", 2, d, L.F, L.enc_emb_W, L.Kp);
  b.vec("encoder.norm.weight", d, L.enc_lng);
  b.vec("encoder.norm.bias", d, L.enc_lnb);
  for (int i = 0; i < L.Le; ++i) enc_block(L.enc[i], "encoder.encoder." + std::to_string(i) + ".");
  b.mat("decoder.word_embedding.weight", L.V, L.dwe, L.emb);
  b.mat("decoder.word_embedding_linear.weight", dd, L.dwe, L.Wel);
  b.vec("decoder.norm.weight", dd, L.dec_lng);
  b.vec("decoder.norm.bias", dd, L.dec_lnb);
  if (L.has_mf) {  // model.py:400-407
    b.mat("decoder.position_wise_1.weight", L.fd, dd, L.mf_W1);
    b.vec("decoder.position_wise_1.bias", L.fd, L.mf_b1);
    b.mat("decoder.position_wise_2.weight", dd, L.fd, L.mf_W2);
    b.vec("decoder.position_wise_2.bias", dd, L.mf_b2);
    b.vec("decoder.layer_norm.weight", dd, L.mf_lng);
    b.vec("decoder.layer_norm.bias", dd, L.mf_lnb);
  }
  for (int i = 0; i < L.Ld; ++i) {
    const auto& e = L.dec[i];
    const std::string p = "decoder.decoder." + std::to_string(i) + ".";
    const std::string s = p + "self_attention.";
    b.mat(s + "q_linear.weight", dd, dd, e.Wqkv);
    b.mat(s + "k_linear.weight", dd, dd, e.Wqkv + dd * dd);
    b.mat(s + "v_linear.weight", dd, dd, e.Wqkv + 2 * dd * dd);
    b.vec(s + "layer_norm.weight", dd, e.lsg);
    b.vec(s + "layer_norm.bias", dd, e.lsb);
    b.mat(s + "joint_linear.weight", dd, dd, e.Wo_s);
    const std::string x = p + "encode_attention.";
    const int64_t kv = L.Wkv_all + (int64_t)i * 2 * dd * d;
    b.mat(x + "q_linear.weight", dd, dd, e.Wq_c);
    b.mat(x + "k_linear.weight", dd, d, kv);
    b.mat(x + "v_linear.weight", dd, d, kv + dd * d);
    b.vec(x + "layer_norm.weight", dd, e.lcg);
    b.vec(x + "layer_norm.bias", dd, e.lcb);
    b.mat(x + "joint_linear.weight", dd, dd, e.Wo_c);
    const std::string f = p + "feed_forward.";
    b.mat(f + "position_wise_1.weight", L.fd, dd, e.W1);
    b.vec(f + "position_wise_1.bias", L.fd, e.b1);
    b.mat(f + "position_wise_2.weight", dd, L.fd, e.W2);
    b.vec(f + "position_wise_2.bias", dd, e.b2);
    b.vec(f + "layer_norm.weight", dd, e.lfg);
    b.vec(f + "layer_norm.bias", dd, e.lfb);
  }
  b.mat("classifer.weight", L.V, dd, L.Wc);  // sic: the reference's attribute name (model.py:68)
  b.vec("classifer.bias", L.V, L.bc);
  return L;
}

}  // namespace capgen
