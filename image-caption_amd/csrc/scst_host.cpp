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
#include <vector>

#include "capgen_host.h"

namespace capgen {
namespace {

constexpr int kN = 4;
constexpr int64_t kDotSentinel = -0x7fffffffffffLL;  // "." when the vocabulary has no such word

// An n-gram of ids.  Two key types with the same interface: a packed uint64 (four 16-bit slots of
// id + 1, zero = unused: vocabularies below 65534 words, integer compares) and the general Gram.
// Counts are vectors sorted by key: a sentence has <= 4 L n-grams, so sorting a small vector and
// merge-joining two of them beats node-based maps (round 1 used std::map<Gram> per sentence).
struct Gram {
  std::array<int64_t, kN> w{};
  int n = 0;
  bool operator<(const Gram& o) const {
    if (n != o.n) return n < o.n;
    return w < o.w;
  }
  bool operator==(const Gram& o) const { return n == o.n && w == o.w; }
};
inline Gram make_gram(const std::vector<int64_t>& t, int i, int k, Gram*) {
  Gram g;
  g.n = k;
  for (int j = 0; j < k; ++j) g.w[j] = t[i + j];
  return g;
}
inline int order_of(const Gram& g) { return g.n; }
inline uint64_t make_gram(const std::vector<int64_t>& t, int i, int k, uint64_t*) {
  uint64_t key = 0;
  for (int j = 0; j < k; ++j) key |= (uint64_t)(t[i + j] + 1) << (16 * (kN - 1 - j));
  return key;
}
inline int order_of(uint64_t key) {
  int n = 0;
  for (int j = 0; j < kN; ++j) n += ((key >> (16 * (kN - 1 - j))) & 0xffff) != 0;
  return n;
}

template <typename K>
using Counts = std::vector<std::pair<K, int>>;

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

template <typename K>
Counts<K> run_counts(std::vector<K>& all) {
  std::sort(all.begin(), all.end());
  Counts<K> c;
  for (const K& g : all) {
    if (!c.empty() && c.back().first == g) ++c.back().second;
    else c.push_back({g, 1});
  }
  return c;
}

template <typename K>
Counts<K> ngrams(const std::vector<int64_t>& t) {
  std::vector<K> all;
  const int len = (int)t.size();
  for (int k = 1; k <= kN; ++k)
    for (int i = 0; i + k <= len; ++i) all.push_back(make_gram(t, i, k, (K*)nullptr));
  return run_counts(all);
}

template <typename K>
struct Vec {
  std::vector<std::pair<K, double>> v[kN];  // sorted by key within each order
  double norm[kN] = {};
  int length = 0;
};

// document frequencies as sorted keys + the idf weight log(#refs) - log(max(1, df)) per key
template <typename K>
struct Df {
  std::vector<K> key;
  std::vector<double> w;
  double w_absent = 0.0;  // an n-gram no reference holds: log(#refs) - log(1)
};

// CiderD._vec: tf * (log(#refs) - log(max(1, df))), per-order norms, length = bigram count
template <typename K>
Vec<K> cider_vec(const Counts<K>& counts, const Df<K>& df) {
  Vec<K> r;
  double sq[kN] = {};
  auto it = df.key.begin();
  for (const auto& kv : counts) {  // both sorted: the search resumes where the last one ended
    it = std::lower_bound(it, df.key.end(), kv.first);
    const double w = it != df.key.end() && *it == kv.first ? df.w[it - df.key.begin()] : df.w_absent;
    const int k = order_of(kv.first) - 1;
    const double x = (double)kv.second * w;
    r.v[k].push_back({kv.first, x});
    sq[k] += x * x;
    if (k == 1) r.length += kv.second;
  }
  for (int k = 0; k < kN; ++k) r.norm[k] = std::sqrt(sq[k]);
  return r;
}

// CiderD._sim (sigma 6): clipped dot product per order, normalised, Gaussian length penalty
template <typename K>
void cider_sim(const Vec<K>& h, const Vec<K>& r, double sigma, double (&val)[kN]) {
  const double delta = (double)(h.length - r.length);
  for (int k = 0; k < kN; ++k) {
    double s = 0.0;
    size_t j = 0;
    for (const auto& kv : h.v[k]) {
      while (j < r.v[k].size() && r.v[k][j].first < kv.first) ++j;
      const double vr = j < r.v[k].size() && r.v[k][j].first == kv.first ? r.v[k][j].second : 0.0;
      s += std::min(kv.second, vr) * vr;
    }
    if (h.norm[k] != 0.0 && r.norm[k] != 0.0) s /= h.norm[k] * r.norm[k];
    val[k] = s * std::exp(-(delta * delta) / (2.0 * sigma * sigma));
  }
}

// Bleu(4) per-sentence score of order 4 against ONE reference ('closest' reference length)
template <typename K>
double bleu4(const std::vector<int64_t>& test, const Counts<K>& tc, const std::vector<int64_t>& ref,
             const Counts<K>& rc) {
  const double tiny = 1e-15, small = 1e-9;
  const int testlen = (int)test.size(), reflen = (int)ref.size();
  int correct[kN] = {}, guess[kN];
  for (int k = 0; k < kN; ++k) guess[k] = std::max(0, testlen - k);
  size_t j = 0;
  for (const auto& kv : tc) {
    while (j < rc.size() && rc[j].first < kv.first) ++j;
    const int m = j < rc.size() && rc[j].first == kv.first ? rc[j].second : 0;
    correct[order_of(kv.first) - 1] += std::min(m, kv.second);
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

template <typename K>
void rewards(const std::vector<std::vector<int64_t>>& ref, const std::vector<std::vector<int64_t>>& hyp, int B,
             double cider_w, double bleu_w, double* out) {
  std::vector<Counts<K>> rc(B), hc(B);
  for (int b = 0; b < B; ++b) rc[b] = ngrams<K>(ref[b]), hc[b] = ngrams<K>(hyp[b]);
  // corpus document frequency: the number of images whose references contain the n-gram
  // (each reference's counts hold every n-gram once: concatenate, sort, count the runs)
  std::vector<K> all;
  for (int b = 0; b < B; ++b)
    for (const auto& kv : rc[b]) all.push_back(kv.first);
  const Counts<K> dfc = run_counts(all);
  const double ref_len = std::log((double)B);
  Df<K> df;
  df.key.reserve(dfc.size());
  df.w.reserve(dfc.size());
  for (const auto& kv : dfc) df.key.push_back(kv.first), df.w.push_back(ref_len - std::log(std::max(1.0, (double)kv.second)));
  df.w_absent = ref_len - std::log(1.0);
  for (int b = 0; b < B; ++b) {
    double cider = 0.0;
    if (cider_w != 0.0) {
      const Vec<K> vh = cider_vec(hc[b], df), vr = cider_vec(rc[b], df);
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

}  // namespace

void scst_rewards(const int64_t* target, int64_t target_ld, const int64_t* sample, int64_t sample_ld, int B, int L,
                  int start_id, int end_id, int null_id, int64_t dot_id, double cider_w, double bleu_w, double* out) {
  require(B >= 1 && L >= 1 && target && sample && out && target_ld >= L && sample_ld >= L,
          "scst_rewards: bad arguments");
  if (dot_id < 0) dot_id = kDotSentinel;
  std::vector<std::vector<int64_t>> ref(B), hyp(B);
  bool packed = true;  // every token id (the "." id included) fits a 16-bit slot as id + 1
  for (int b = 0; b < B; ++b) {
    ref[b] = tokens(target + (int64_t)b * target_ld, L, start_id, end_id, null_id, dot_id);
    hyp[b] = tokens(sample + (int64_t)b * sample_ld, L, start_id, end_id, null_id, dot_id);
    for (const auto* t : {&ref[b], &hyp[b]})
      for (int64_t id : *t) packed = packed && id >= 0 && id < 0xfffe;
  }
  if (!packed && dot_id == kDotSentinel) {  // the sentinel is the only out-of-range id: give it 0xfffe
    bool others = true;
    for (int b = 0; b < B; ++b)
      for (const auto* t : {&ref[b], &hyp[b]})
        for (int64_t id : *t) others = others && (id == kDotSentinel || (id >= 0 && id < 0xfffe));
    if (others) {
      for (int b = 0; b < B; ++b)
        for (auto* t : {&ref[b], &hyp[b]})
          for (int64_t& id : *t)
            if (id == kDotSentinel) id = 0xfffe;
      packed = true;
    }
  }
  if (packed) rewards<uint64_t>(ref, hyp, B, cider_w, bleu_w, out);
  else rewards<Gram>(ref, hyp, B, cider_w, bleu_w, out);
}

}  // namespace capgen
