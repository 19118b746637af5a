// Host-only C++ of libcapgen under AddressSanitizer + UBSan (make -C image-caption_amd/csrc asan;
// run by tests/test_asan.py): the persisted tune-table line parser, the parameter-arena layout and
// its reference-name table, the SCST n-gram scorer and the run-time switch registry, fed valid,
// adversarial and random inputs.  Exit status 0 = every check held and the sanitizers saw nothing.
//   asan_host <tune table path>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "../image-caption_amd/csrc/capgen_host.h"
#include "../image-caption_amd/csrc/layout.h"
#include "../image-caption_amd/csrc/tune_parse.h"

namespace capgen {
void scst_rewards(const int64_t* target, int64_t target_ld, const int64_t* sample, int64_t sample_ld, int B, int L,
                  int start_id, int end_id, int null_id, int64_t dot_id, double cider_w, double bleu_w, double* out);
}

using namespace capgen;

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

static void tune_lines(const char* path) {
  const int allowed[] = {6, 20, 17, 18, 19, 4, 8, 1, 3, 10};
  int good = 0;
  std::ifstream f(path);
  std::string line;
  while (std::getline(f, line)) {
    if (line.empty()) continue;
    TuneLineG g;
    std::vector<int> key;
    int var = 0;
    if (line[0] == 'g') good += parse_tune_g(line.c_str() + 1, 27, &g);
    if (line[0] == 'G') good += parse_tune_G(line.c_str() + 1, allowed, 10, 8, &key, &var);
  }
  CHECK(good > 50);  // the committed table parses
  // adversarial lines: truncated, overlong, out-of-range counts, garbage, a huge group count
  const char* bad[] = {"", " ", "1 2 3", " 1 2 3 4 5 6 7", " 1 2 3 4 5 6 99 1", " 1 2 3 4 5 6 7 0", " a b c",
                       " 1 1 4 9 1 2 3 10", " 1 1 4 -5 1 2 3 10", " 1 1 4 1000000 1 2 3 10", " 1 1 4 1 1 2 3",
                       " 99999999999999999999 1 2 3 4 5 6 7"};
  for (const char* b : bad) {
    TuneLineG g;
    std::vector<int> key;
    int var = 0;
    CHECK(!parse_tune_g(b, 27, &g));
    (void)parse_tune_G(b, allowed, 10, 8, &key, &var);
  }
  std::string longline(" 1 1 4 8");
  for (int i = 0; i < 500; ++i) longline += " 7";
  std::vector<int> key;
  int var = 0;
  CHECK(!parse_tune_G(longline.c_str(), allowed, 10, 8, &key, &var));
  TuneLineG g;
  CHECK(parse_tune_g(" 2304 512 2048 0 1 2 7 1  # 64x64w4s3", 27, &g) && g.K == 2048 && g.variant == 7);
  CHECK(parse_tune_G(" 1 1 4 1 512 2048 1216 10  # x", allowed, 10, 8, &key, &var) && var == 10 && key.size() == 6);
}

static capgen_config base(int d, int ff, int le, int ld, int h, int V, int F, int P) {
  capgen_config c;
  std::memset(&c, 0, sizeof c);
  c.num_vocab = V, c.max_length = 20, c.dim_features = F, c.dim_positions = P;
  c.enc_d = d, c.enc_ff = ff, c.enc_blocks = le, c.enc_heads = h, c.dim_word_embedding = d;
  c.dec_d = d, c.dec_ff = ff, c.dec_blocks = ld, c.dec_heads = h;
  c.dropout = 0.3f, c.attention_dropout = 0.1f, c.dtype = CAPGEN_BF16, c.max_batch = 64, c.max_regions = 36;
  c.lr = 5e-4f, c.beta1 = 0.9f, c.beta2 = 0.999f, c.eps = 1e-8f;
  return c;
}

static void layouts() {
  std::vector<capgen_config> cs;
  cs.push_back(base(128, 512, 2, 2, 4, 1000, 512, 84));
  cs.push_back(base(512, 2048, 6, 6, 8, 10000, 2048, 84));
  for (int flag = 0; flag < 5; ++flag) {
    capgen_config c = base(128, 512, 2, 2, 4, 1000, 512, 84);
    if (flag == 0) c.encode_mask = 1;
    if (flag == 1) c.focal_loss = 1;
    if (flag == 2) c.split_position = 1;
    if (flag == 3) c.split_image_objects = 1;
    if (flag == 4) c.move_first_image_feature = 1;
    cs.push_back(c);
  }
  for (const auto& c : cs) {
    Layout L = make_layout(c);
    CHECK(L.total > 0 && L.n_dense > 0 && L.n_dense <= L.total && !L.table.empty());
    for (const auto& p : L.table) {
      CHECK(std::strlen(p.name) > 0 && std::strlen(p.name) < sizeof p.name);
      CHECK(p.offset >= 0 && p.offset + (p.rows - 1) * p.row_stride + p.cols <= L.total);
    }
  }
  // invalid configurations are refused with an Error, not undefined behaviour
  capgen_config bad = base(128, 512, 2, 2, 4, 1000, 512, 84);
  bad.split_position = bad.split_image_objects = 1;
  bool threw = false;
  try {
    (void)make_layout(bad);
  } catch (const Error&) {
    threw = true;
  }
  CHECK(threw);
  bad = base(100, 512, 2, 2, 4, 1000, 512, 84);
  threw = false;
  try {
    (void)make_layout(bad);
  } catch (const Error&) {
    threw = true;
  }
  CHECK(threw);
}

static void scst() {
  std::mt19937_64 rng(7);
  for (int trial = 0; trial < 6; ++trial) {
    const int B = 1 + (int)(rng() % 64), L = 1 + (int)(rng() % 20);
    const int64_t V = trial == 3 ? (int64_t)1 << 20 : 10000;  // trial 3: ids past the packed 16-bit form
    std::vector<int64_t> t((size_t)B * L), s((size_t)B * L);
    for (auto* v : {&t, &s})
      for (auto& x : *v) x = (int64_t)(rng() % V);
    if (trial == 2)
      for (auto& x : s) x = 0;  // every sample empty (<NULL>)
    std::vector<double> out(B, -1.0);
    scst_rewards(t.data(), L, s.data(), L, B, L, 1, 2, 0, trial % 2 ? -1 : 3, 1.0, 0.5, out.data());
    for (double r : out) CHECK(r >= 0.0 && r == r);
    scst_rewards(t.data(), L, t.data(), L, B, L, 1, 2, 0, -1, 1.0, 0.0, out.data());
    for (double r : out) CHECK(r >= 0.0);
  }
  bool threw = false;
  try {
    double o;
    scst_rewards(nullptr, 1, nullptr, 1, 1, 1, 1, 2, 0, -1, 1.0, 0.0, &o);
  } catch (const Error&) {
    threw = true;
  }
  CHECK(threw);
}

static void knobs() {
  int old = -7;
  CHECK(knob(Knob::FusedCe) == 1);
  CHECK(knob_set("FUSED_CE", 0, &old) == 0 && old == 1 && knob(Knob::FusedCe) == 0);
  CHECK(knob_set("FUSED_CE", 1, nullptr) == 0);
  CHECK(knob_set("NO_SUCH_SWITCH", 1, &old) == -1);
  CHECK(knob_set("SKIP", 1, &old) == -2 && knob(Knob::Skip) == 0);  // debug-only in a product build
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: asan_host <tune table>\n");
    return 2;
  }
  tune_lines(argv[1]);
  layouts();
  scst();
  knobs();
  std::printf("asan_host: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
