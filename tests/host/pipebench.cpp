// pipebench.cpp -- host-side cost of the cross-height pipeline (plan, pack,
// replay) without a device: commit.cpp + pipeline.cpp over
// tests/host/fake_runtime.cpp with every verdict valid and nothing decoded.
// configs[2]'s shape: n_heights commits x 150 validators, all signatures
// present, one validator set (registered keys). Prints ms per call.
// Usage: pipebench [n_heights] [threads] [kind] [chunk] [n_vals] [pipe] [single] [devices] [pinned]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/cmtverify.h"

extern "C" {
cmtv_ctx* fake_open(size_t n_devs, unsigned threads, size_t pipe_min, size_t chunk, int slots, bool pipe_on,
                    size_t keyset_cap, long fail_dev);
void fake_set_noverify(cmtv_ctx* c, bool on);
void fake_phases(cmtv_ctx* c, uint64_t* out);
void fake_close(cmtv_ctx* c);
void fake_counts(cmtv_ctx* c, uint64_t* out);
}

int main(int argc, char** argv) {
  const size_t H = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000;
  const unsigned T = argc > 2 ? (unsigned)std::atoi(argv[2]) : 8;
  const uint32_t kind = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 0;
  const size_t chunk = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : (1u << 20);
  const uint32_t nv = argc > 5 ? (uint32_t)std::atoi(argv[5]) : 150;
  const bool pipe = argc > 6 ? std::atoi(argv[6]) != 0 : true;
  std::vector<uint8_t> pk(32 * nv), addrs(20 * nv + 1);
  std::vector<uint32_t> pk_off(nv + 1);
  std::vector<int64_t> power(nv, 10), prio(nv, 0);
  for (uint32_t i = 0; i < nv; i++) {
    for (int k = 0; k < 32; k++) pk[32 * i + k] = (uint8_t)(i * 7 + k);
    std::memcpy(&addrs[20 * i], &pk[32 * i], 20);
  }
  for (uint32_t i = 0; i <= nv; i++) pk_off[i] = 32 * i;
  cmtv_valset vs{nv, pk.data(), pk_off.data(), power.data(), addrs.data(), prio.data()};
  // argv[8]: fake devices (chunks round-robin over their lanes, as on a node);
  // argv[9] = 1 (default): the commits' flags, timestamps and signatures in
  // ONE cmtv_alloc_pinned block (class arrays, as tests/host/pipecheck.cpp
  // kClassArrays) -- the direct chunks; 0: heap memory, every chunk packed
  const size_t devs = argc > 8 ? std::strtoull(argv[8], nullptr, 10) : 1;
  const bool pinned = argc > 9 ? std::atoi(argv[9]) != 0 : true;
  cmtv_ctx* ctx = fake_open(devs, T, 1, chunk, 3, pipe, 4, -1);
  const size_t n_sig = (size_t)nv * H;
  std::vector<uint8_t> heap;
  uint8_t* arena = nullptr;
  const size_t arena_bytes = 64 + (nv + 1) + 8 * n_sig + 4 * nv + 64 * n_sig + 256;
  if (pinned) {
    if (cmtv_alloc_pinned(ctx, arena_bytes, reinterpret_cast<void**>(&arena)) != CMTV_OK) return 2;
  } else {
    heap.resize(arena_bytes + 64);
    arena = heap.data() + (64 - (reinterpret_cast<uintptr_t>(heap.data()) & 63));
  }
  uint8_t* flags = arena;
  auto* secs = reinterpret_cast<int64_t*>(arena + 256);
  auto* nanos = reinterpret_cast<int32_t*>(reinterpret_cast<uint8_t*>(secs) + 8 * n_sig);
  uint8_t* sigs = reinterpret_cast<uint8_t*>(nanos) + 4 * ((nv + 15) / 16 * 16);
  std::memset(flags, 2, nv + 1);
  std::vector<uint8_t> bh(32 * H), ph(32 * H);
  std::vector<uint32_t> sig_off(nv + 1);
  for (uint32_t i = 0; i <= nv; i++) sig_off[i] = 64 * i;
  for (uint32_t i = 0; i < nv; i++) nanos[i] = (int32_t)(i * 1000);
  for (size_t i = 0; i < 64 * n_sig; i++) sigs[i] = (uint8_t)(i * 131 + (i >> 9));
  std::vector<cmtv_commit> cs(H);
  std::vector<cmtv_block_id> bids(H);
  std::vector<cmtv_valset> vals(H, vs);
  std::vector<int64_t> hs(H);
  for (size_t h = 0; h < H; h++) {
    for (int k = 0; k < 32; k++) {
      bh[32 * h + k] = (uint8_t)(h + k);
      ph[32 * h + k] = (uint8_t)(h * 3 + k);
    }
    for (uint32_t i = 0; i < nv; i++) secs[nv * h + i] = 1672531200 + (int64_t)h;
    bids[h] = cmtv_block_id{&bh[32 * h], 32, 1, &ph[32 * h], 32};
    hs[h] = (int64_t)h + 1;
    cs[h] = cmtv_commit{(int64_t)h + 1, 0, bids[h], nv, flags, &secs[nv * h], nanos, &sigs[64 * nv * h],
                        sig_off.data(), addrs.data()};
  }
  std::vector<cmtv_commit_result> res(H);
  std::vector<int> rcs(H);
  fake_set_noverify(ctx, true);
  const char chain[] = "cmtverify-bench";
  double best = 1e30;
  uint64_t pt0[16] = {};
  // argv[7] = 1: the single-commit entry point (cmtv_verify_commit on
  // commit 0) instead, its host cost per call
  const bool single = argc > 7 && std::atoi(argv[7]) != 0;
  const int iters = single ? 20000 : H == 1 ? 200 : 6;
  for (int it = 0; it < iters; it++) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = single ? cmtv_verify_commit(ctx, kind, 0, chain, sizeof chain - 1, &vals[0], &bids[0], hs[0], &cs[0],
                                               1, 3, &res[0], nullptr, 0)
                          : cmtv_verify_commits(ctx, kind, 0, chain, sizeof chain - 1, H, vals.data(), bids.data(),
                                                hs.data(), cs.data(), 1, 3, res.data(), rcs.data(), nullptr, 0);
    if (single) rcs[0] = rc;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc != CMTV_OK || rcs[0] != 0) {
      std::fprintf(stderr, "rc %d rcs[0] %d\n", rc, rcs[0]);
      return 1;
    }
    if (it) best = ms < best ? ms : best;
    if (it == 0) fake_phases(ctx, pt0);  // the phases below leave out the warm-up call (first touch)
  }
  uint64_t cnt[6];
  fake_counts(ctx, cnt);
  std::printf("%zu heights x %u, kind %u, %u threads, %zu devices, %s, %s (%llu direct chunks): %.4f ms per call (%.1f ns per signature of wall)\n", H, nv, kind,
              T, devs, pipe ? "pipeline" : "one batch", pinned ? "pinned arena" : "heap", (unsigned long long)cnt[5], best, best * 1e6 / (double)(H * nv));
  uint64_t pt[16] = {};
  fake_phases(ctx, pt);
  for (int p = 0; p < 16; p++) pt[p] -= pt0[p];
  const double k = 1e6 * (iters - 1);
  std::printf("  per call ms: plan %.3f pack %.3f submit %.3f wait %.3f replay %.3f cut %.3f | one batch: prepare %.4f "
              "replay %.4f\n", pt[6] / k, pt[7] / k, pt[8] / k, pt[9] / k, pt[10] / k, pt[13] / k, pt[0] / k, pt[5] / k);
  fake_close(ctx);
  return 0;
}
