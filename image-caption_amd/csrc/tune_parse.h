// capgen — line parser of the persisted GEMM autotune table (host only; gemm_bf16.hip loads the
// table through it, tests/asan_host.cpp drives it under AddressSanitizer).
//   g M N K ta tb out_bytes variant splitk  [# comment]
//   G ta tb out_bytes n (M N K) x n variant  [# comment]
#pragma once
#include <vector>

namespace capgen {

struct TuneLineG {
  int M = 0, N = 0, K = 0, ta = 0, tb = 0, out = 0, variant = 0, splitk = 0;
};
// a 'g' line (text after the 'g'): true with every field read, M / N / K >= 1, ta / tb in {0, 1}, out_bytes
// in {2, 4}, variant in [1, nvariants], split-K in [1, 16]
bool parse_tune_g(const char* rest, int nvariants, TuneLineG* out);
// a 'G' line (text after the 'G'): true with ta / tb in {0, 1}, out_bytes in {2, 4}, n in [1, max_group],
// exactly 3 n positive shape numbers and a variant from `allowed`; key = {ta, tb, out_bytes, M0, N0, K0, M1, ...}
bool parse_tune_G(const char* rest, const int* allowed, int n_allowed, int max_group, std::vector<int>* key,
                  int* variant);

}  // namespace capgen
