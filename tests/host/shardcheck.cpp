// Host build of cometbft_amd/csrc/shard.h: reads (n, devices, shard_min)
// triples (3 x u64) on stdin, writes (G, S, W) per triple. Test
// infrastructure only (tests/test_shard_plan.py checks the invariants).
#include <cstdint>
#include <cstdio>

#include "../../cometbft_amd/csrc/shard.h"

int main() {
  uint64_t t[3];
  while (fread(t, 8, 3, stdin) == 3) {
    const cmtv::ShardPlan p = cmtv::plan_shards(t[0], t[1], t[2]);
    const uint64_t o[3] = {p.G, p.S, p.W};
    fwrite(o, 8, 3, stdout);
  }
  return 0;
}
