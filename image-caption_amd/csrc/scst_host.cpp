// capgen — native host rewards for self-critical training: CIDEr-D (corpus document
// frequencies) + per-sentence BLEU-4 over token ids, the arithmetic of capgen/scst.py
// (CiderD.compute_score, Bleu.compute_score; StructureCriterion.get_scores, loss.py:154-181)
// without the Python dict/string work (~7 ms per 64-image step there, tools/bench_scst.py).
//
// Sentences are compared as token-id sequences: decode_captions (core/utils.py:67-103)
// maps ids to words one to one (skip <START> at t = 0, <END> -> "." and stop, drop <NULL>),
// so n-gram statistics over ids equal those over words when "." is given the id of the
// vocabulary's "." word (or a sentinel when it has none).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <map>
#include <vector>

#include "capgen_common.h"

namespace capgen {
namespace {

constexpr int kN = 4;
constexpr int64_t kDotSentinel = -0x7fffffffffffLL;  // "." when the vocabulary has no such word

// an n-gram of ids (order = number of valid entries)
struct Gram {
  std::array<int64_t, kN> w{};
  int n = 0;
  bool operator<(const Gram& o) const {
    if (n != o.n) return n < o.n;
    return w < o.w;
  }
};
typedef std::map<Gram, int> Counts;

std::vector<int64_t> tokens(const int64_t* row, int L, int start_id, int end_id, int null_id, int64_t dot_id) {
  std::vector<int64_t> t;
  for (int i = 0; i < L; ++i) {
    const int64_t id = row[i];
    if (id == start_id && i == 0) continue;
    if (id == end_id) {
      t.push_back(dot_id);
      break;
    }
    if (id != null_id) t.push_back(id);
  }
  return t;
}

Counts ngrams(const std::vector<int64_t>& t) {
  Counts c;
  const int len = (int)t.size();
  for (int k = 1; k <= kN; ++k)
    for (int i = 0; i + k <= len; ++i) {
      Gram g;
      g.n = k;
      for (int j = 0; j < k; ++j) g.w[j] = t[i + j];
      ++c[g];
    }
  return c;
}

struct Vec {
  std::map<Gram, double> v[kN];
  double norm[kN] = {};
  int length = 0;
};

// CiderD._vec: tf * (log(#refs) - log(max(1, df))), per-order norms, length = bigram count
Vec cider_vec(const Counts& counts, const std::map<Gram, int>& df, double ref_len) {
  Vec r;
  double sq[kN] = {};
  for (const auto& kv : counts) {
    const int k = kv.first.n - 1;
    auto it = df.find(kv.first);
    const double d = it == df.end() ? 0.0 : (double)it->second;
    const double x = (double)kv.second * (ref_len - std::log(std::max(1.0, d)));
    r.v[k][kv.first] = x;
    sq[k] += x * x;
    if (k == 1) r.length += kv.second;
  }
  for (int k = 0; k < kN; ++k) r.norm[k] = std::sqrt(sq[k]);
  return r;
}

// CiderD._sim (sigma 6): clipped dot product per order, normalised, Gaussian length penalty
void cider_sim(const Vec& h, const Vec& r, double sigma, double (&val)[kN]) {
  const double delta = (double)(h.length - r.length);
  for (int k = 0; k < kN; ++k) {
    double s = 0.0;
    for (const auto& kv : h.v[k]) {
      auto it = r.v[k].find(kv.first);
      const double vr = it == r.v[k].end() ? 0.0 : it->second;
      s += std::min(kv.second, vr) * vr;
    }
    if (h.norm[k] != 0.0 && r.norm[k] != 0.0) s /= h.norm[k] * r.norm[k];
    val[k] = s * std::exp(-(delta * delta) / (2.0 * sigma * sigma));
  }
}

// Bleu(4) per-sentence score of order 4 against ONE reference ('closest' reference length)
double bleu4(const std::vector<int64_t>& test, const Counts& tc, const std::vector<int64_t>& ref, const Counts& rc) {
  const double tiny = 1e-15, small = 1e-9;
  const int testlen = (int)test.size(), reflen = (int)ref.size();
  int correct[kN] = {}, guess[kN];
  for (int k = 0; k < kN; ++k) guess[k] = std::max(0, testlen - k);
  for (const auto& kv : tc) {
    auto it = rc.find(kv.first);
    const int m = it == rc.end() ? 0 : it->second;
    correct[kv.first.n - 1] += std::min(m, kv.second);
  }
  double b = 1.0, out = 0.0;
  for (int k = 0; k < kN; ++k) {
    b *= (correct[k] + tiny) / (guess[k] + small);
    out = std::pow(b, 1.0 / (k + 1));
  }
  const double ratio = (testlen + tiny) / (reflen + small);
  if (ratio < 1.0) out *= std::exp(1.0 - 1.0 / ratio);
  return out;
}

}  // namespace

void scst_rewards(const int64_t* target, int64_t target_ld, const int64_t* sample, int64_t sample_ld, int B, int L,
                  int start_id, int end_id, int null_id, int64_t dot_id, double cider_w, double bleu_w, double* out) {
  require(B >= 1 && L >= 1 && target && sample && out && target_ld >= L && sample_ld >= L,
          "scst_rewards: bad arguments");
  if (dot_id < 0) dot_id = kDotSentinel;
  std::vector<std::vector<int64_t>> ref(B), hyp(B);
  std::vector<Counts> rc(B), hc(B);
  for (int b = 0; b < B; ++b) {
    ref[b] = tokens(target + (int64_t)b * target_ld, L, start_id, end_id, null_id, dot_id);
    hyp[b] = tokens(sample + (int64_t)b * sample_ld, L, start_id, end_id, null_id, dot_id);
    rc[b] = ngrams(ref[b]);
    hc[b] = ngrams(hyp[b]);
  }
  // corpus document frequency: the number of images whose references contain the n-gram
  std::map<Gram, int> df;
  for (int b = 0; b < B; ++b)
    for (const auto& kv : rc[b]) ++df[kv.first];
  const double ref_len = std::log((double)B);
  for (int b = 0; b < B; ++b) {
    double cider = 0.0;
    if (cider_w != 0.0) {
      const Vec vh = cider_vec(hc[b], df, ref_len), vr = cider_vec(rc[b], df, ref_len);
      double val[kN];
      cider_sim(vh, vr, 6.0, val);
      double acc = 0.0;
      for (int k = 0; k < kN; ++k) acc += val[k];
      cider = acc / kN * 10.0;  // mean over orders, one reference, x10
    }
    const double bleu = bleu_w != 0.0 ? bleu4(hyp[b], hc[b], ref[b], rc[b]) : 0.0;
    out[b] = cider_w * cider + bleu_w * bleu;
  }
}

}  // namespace capgen
