// shard.h -- how a host batch is split across the devices of a context
// (runtime.cpp). Plain C++, shared with the host test
// tests/host/shardcheck.cpp.
//
// G devices take contiguous shards of S signatures each, S a multiple of 64,
// so shard g's verdict bits start at bitmap word g * S / 64 and the shards'
// bitmaps concatenate into the batch's bitmap with no repacking (the RCCL
// all-gather is in place). The last shards may be short or empty.
//
// A device's share is at least shard_min signatures (below that one device
// runs its share in a single kernel-chain time anyway, so a further split
// only adds staging and a gather): a batch uses
//     G = min(n_devs, max(1, floor(n / max(shard_min, 64))))
// devices, the first G of the context's usable devices -- a 40k batch with
// shard_min 8192 runs on 4 of 8 GPUs, not on one.
#pragma once
#include <stddef.h>

#include <algorithm>

namespace cmtv {

struct ShardPlan {
  size_t G = 1;  // devices used
  size_t S = 0;  // signatures per shard (a multiple of 64 when G > 1)
  size_t W = 0;  // bitmap words per shard
  size_t lo(size_t g, size_t n) const { return std::min(n, g * S); }
  size_t hi(size_t g, size_t n) const { return std::min(n, (g + 1) * S); }
};

inline ShardPlan plan_shards(size_t n, size_t n_devs, size_t shard_min) {
  ShardPlan p;
  const size_t per = std::max<size_t>(shard_min, 64);
  size_t G = n_devs ? n_devs : 1;
  G = std::min(G, std::max<size_t>(1, n / per));
  p.G = G;
  p.S = G == 1 ? n : ((n + G - 1) / G + 63) / 64 * 64;
  p.W = (p.S + 63) / 64;
  return p;
}

}  // namespace cmtv
