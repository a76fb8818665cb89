// Host build of cometbft_amd/csrc/halfscalar.h (the device source): reads
// n x 32-byte little-endian scalars k on stdin, writes per scalar
// k1 (32 B) | |k2| (32 B) | flags (1 B: bit0 k2 negative, bit1 wide,
// bits 2-7 the window count - 32),
// twice: Lehmer schedule, then exact single steps. argv[1] == "any": the
// ZIP-215 choice (k2 of any parity), else k2 odd (GO_STDLIB). Test
// infrastructure only (tests/test_host_math.py checks the invariants).
#define CMTV_HD inline
#include <cstdio>
#include <initializer_list>
#include "../../cometbft_amd/csrc/halfscalar.h"

int main(int argc, char** argv) {
  const bool odd = !(argc > 1 && argv[1][0] == 'a');
  uint32_t n;
  if (fread(&n, 4, 1, stdin) != 1) return 1;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t k[8];
    if (fread(k, 4, 8, stdin) != 8) return 1;
    cmtv::HalfScalars h, g;
    cmtv::half_scalars<true>(h, k, false, odd);   // Lehmer rounds (the device schedule)
    cmtv::half_scalars<false>(g, k, false, odd);  // one exact Euclid step per round
    for (const cmtv::HalfScalars* x : {&h, &g}) {
      uint8_t f = (x->k2_neg ? 1 : 0) | (x->wide ? 2 : 0) | (uint8_t)((x->windows - 32) << 2);
      fwrite(x->k1, 4, 8, stdout);
      fwrite(x->k2, 4, 8, stdout);
      fwrite(&f, 1, 1, stdout);
    }
  }
  return 0;
}
