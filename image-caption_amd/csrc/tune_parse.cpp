// capgen — persisted autotune table lines (tune_parse.h).
#include "tune_parse.h"

#include <algorithm>
#include <cstdio>

namespace capgen {

bool parse_tune_g(const char* rest, int nvariants, TuneLineG* o) {
  TuneLineG k;
  if (std::sscanf(rest, "%d %d %d %d %d %d %d %d", &k.M, &k.N, &k.K, &k.ta, &k.tb, &k.out, &k.variant, &k.splitk) != 8)
    return false;
  if (k.M < 1 || k.N < 1 || k.K < 1 || (k.ta != 0 && k.ta != 1) || (k.tb != 0 && k.tb != 1) ||
      (k.out != 2 && k.out != 4) || k.variant < 1 || k.variant > nvariants || k.splitk < 1 || k.splitk > 16)
    return false;
  *o = k;
  return true;
}

bool parse_tune_G(const char* rest, const int* allowed, int n_allowed, int max_group, std::vector<int>* key,
                  int* variant) {
  std::vector<int> v;
  const char* p = rest;
  int x = 0, used = 0;
  while (v.size() < 64 && std::sscanf(p, "%d%n", &x, &used) == 1) v.push_back(x), p += used;
  if (v.size() < 5) return false;
  if (std::find(allowed, allowed + n_allowed, v.back()) == allowed + n_allowed) return false;
  // (a stale or corrupt variant is skipped: the group is tuned again)
  if (v[3] < 1 || v[3] > max_group || v.size() != 4 + 3 * (size_t)v[3] + 1) return false;
  if ((v[0] != 0 && v[0] != 1) || (v[1] != 0 && v[1] != 1) || (v[2] != 2 && v[2] != 4)) return false;
  for (int i = 0; i < 3 * v[3]; ++i)
    if (v[4 + i] < 1) return false;
  key->assign({v[0], v[1], v[2]});
  key->insert(key->end(), v.begin() + 4, v.end() - 1);
  *variant = v.back();
  return true;
}

}  // namespace capgen
