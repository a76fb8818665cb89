// shard.h -- how a host batch is split across the devices of a context
// (runtime.cpp). Plain C++, shared with the host test
// tests/host/shardcheck.cpp.
//
// G devices take contiguous shards of S signatures each, S a multiple of 64,
// so shard g's verdict bits start at bitmap word g * S / 64 and the shards'
// bitmaps concatenate into the batch's bitmap with no repacking (the RCCL
// all-gather is in place). The last shards may be short or empty. Batches of
// fewer than shard_min signatures per device stay on device 0: below that a
// device's share runs in one kernel-chain time anyway, so splitting only adds
// staging and a gather.
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
  size_t G = n_devs ? n_devs : 1;
  if (G > 1 && n < G * std::max<size_t>(shard_min, 64)) G = 1;
  p.G = G;
  p.S = G == 1 ? n : ((n + G - 1) / G + 63) / 64 * 64;
  p.W = (p.S + 63) / 64;
  return p;
}

}  // namespace cmtv
