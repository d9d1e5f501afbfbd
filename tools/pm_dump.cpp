// Dumps the merged partial-round tables the device code uses (csrc/poseidon.h make_pm) as JSON,
// for tests/test_poseidon_merge.py to compare with its exact-integer model.  Host build only:
//   g++ -std=c++17 -O1 -o pm_dump tools/pm_dump.cpp
#include <cstdio>
#include "../plonky2-verifier_amd/csrc/poseidon.h"

int main() {
  static const p2::PMTab T = p2::make_pm();
  std::printf("{\"sched\": [");
  for (int b = 0; b < p2::PM_NB; b++) std::printf("%s%d", b ? ", " : "", p2::PM_SCHED[b]);
  std::printf("], \"blocks\": [");
  for (int b = 0; b < p2::PM_NB; b++) {
    const p2::PBlock& B = T.b[b];
    std::printf("%s{\"cf\": [", b ? ", " : "");
    for (int r = 0; r < 14; r++) {
      std::printf("%s[", r ? ", " : "");
      for (int j = 0; j < 16; j++) std::printf("%s%u", j ? ", " : "", B.cf[r][j]);
      std::printf("]");
    }
    std::printf("], \"d\": [");
    for (int k = 0; k < 16; k++) std::printf("%s%llu", k ? ", " : "", (unsigned long long)((B.dhi[k] << 32) | B.dlo[k]));
    std::printf("]}");
  }
  std::printf("]}\n");
  return 0;
}
