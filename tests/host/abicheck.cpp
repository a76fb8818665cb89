// Sanitizer driver for the host side of libcmtverify (runtime.cpp,
// commit.cpp): built with host-only AddressSanitizer + UBSan
// (cometbft_amd/csrc/Makefile target `san`), linked with the same gfx950
// kernel objects, and driven through the public C ABI only. Test
// infrastructure (tests/test_sanitizers.py).
//
//   abicheck <vectors.bin> [threads]
// vectors.bin: u32 n, then n x { pk[32], sig[64], u32 mlen, msg[mlen], u8 go, u8 zip215 }.
// Without a device it checks the ENODEV path and the device-free entry
// points; with one it verifies the vectors in both modes (single-device,
// a sharded context over a repeated ordinal, the BatchVerifier mirror, a
// commit replay) and runs `threads` concurrent callers on one context.
// Exit 0 = every check passed.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cmtverify.h"

static int fails = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      fails++;                                                      \
    }                                                               \
  } while (0)

struct Vecs {
  size_t n = 0;
  std::vector<uint8_t> pk, sig, msg, go, zip;
  std::vector<uint32_t> off{0};
};

static bool load(const char* path, Vecs& v) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  uint32_t n;
  if (std::fread(&n, 4, 1, f) != 1) return false;
  v.n = n;
  v.pk.resize(32 * n);
  v.sig.resize(64 * n);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t ml;
    uint8_t e[2];
    if (std::fread(&v.pk[32 * i], 32, 1, f) != 1 || std::fread(&v.sig[64 * i], 64, 1, f) != 1 ||
        std::fread(&ml, 4, 1, f) != 1)
      return false;
    const size_t o = v.msg.size();
    v.msg.resize(o + ml);
    if (ml && std::fread(&v.msg[o], ml, 1, f) != 1) return false;
    if (std::fread(e, 2, 1, f) != 1) return false;
    v.go.push_back(e[0]);
    v.zip.push_back(e[1]);
    v.off.push_back((uint32_t)v.msg.size());
  }
  std::fclose(f);
  if (v.msg.empty()) v.msg.push_back(0);
  return true;
}

static void device_free_checks() {
  CHECK(std::strcmp(cmtv_strerror(CMTV_EINVAL), "invalid argument") == 0);
  CHECK(cmtv_abi_version() == CMTV_ABI_VERSION);
  cmtv_ctx* c = nullptr;
  CHECK(cmtv_open(nullptr, nullptr) == CMTV_EINVAL);
  CHECK(cmtv_open_devices(nullptr, nullptr, 0, nullptr) == CMTV_EINVAL);
  CHECK(cmtv_verify_ed25519(nullptr, 1, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr) == CMTV_EINVAL);
  CHECK(cmtv_sync(nullptr) == CMTV_EINVAL);
  (void)c;
  // sign-bytes: types/vote_test.go:60-137 vector #3 (type 1, height 1, round 1, zero time)
  uint8_t out[256];
  const int64_t n = cmtv_vote_sign_bytes(nullptr, 0, 1, 1, 1, nullptr, -62135596800LL, 0, out, sizeof out);
  const uint8_t want[] = {0x21, 0x08, 0x01, 0x11, 0x01, 0, 0, 0, 0, 0, 0, 0, 0x19, 0x01, 0, 0, 0, 0, 0, 0,
                          0, 0x2a, 0x0b, 0x08, 0x80, 0x92, 0xb8, 0xc3, 0x98, 0xfe, 0xff, 0xff, 0xff, 0x01};
  CHECK(n == (int64_t)sizeof want && std::memcmp(out, want, sizeof want) == 0);
  // length query with a short buffer
  CHECK(cmtv_vote_sign_bytes("chain", 5, 2, 7, 0, nullptr, 1, 2, out, 3) > 3);
}

static bool verify_eq(cmtv_ctx* ctx, const Vecs& v, uint32_t mode) {
  std::vector<uint8_t> got(v.n);
  std::vector<uint64_t> bm((v.n + 63) / 64);
  if (cmtv_verify_ed25519(ctx, v.n, v.pk.data(), v.sig.data(), v.msg.data(), v.off.data(), mode, got.data(),
                          bm.data()) != CMTV_OK)
    return false;
  const auto& exp = mode ? v.zip : v.go;
  for (size_t i = 0; i < v.n; i++)
    if (got[i] != exp[i] || (((bm[i / 64] >> (i % 64)) & 1) != exp[i])) return false;
  return true;
}

static void device_checks(const Vecs& v, int threads) {
  cmtv_ctx* ctx = nullptr;
  cmtv_config cfg{0, CMTV_MODE_GO_STDLIB, 0, 0};
  CHECK(cmtv_open(&cfg, &ctx) == CMTV_OK);
  if (!ctx) return;
  CHECK(verify_eq(ctx, v, CMTV_MODE_GO_STDLIB));
  CHECK(verify_eq(ctx, v, CMTV_MODE_ZIP215));
  // BatchVerifier mirror: bad signature / key lengths, reset, reuse
  cmtv_batch* b = nullptr;
  CHECK(cmtv_batch_new(ctx, CMTV_MODE_GO_STDLIB, &b) == CMTV_OK);
  for (size_t i = 0; i < v.n; i++)
    CHECK(cmtv_batch_add(b, &v.pk[32 * i], 32, &v.msg[v.off[i]], v.off[i + 1] - v.off[i], &v.sig[64 * i], 64) == 0);
  CHECK(cmtv_batch_add(b, v.pk.data(), 31, v.msg.data(), 1, v.sig.data(), 64) == 0);
  CHECK(cmtv_batch_add(b, v.pk.data(), 32, v.msg.data(), 1, v.sig.data(), 63) == 0);
  std::vector<uint8_t> out(cmtv_batch_len(b));
  int all_ok = 1;
  int64_t bad_key = -2;
  CHECK(cmtv_batch_verify(b, out.data(), &all_ok, &bad_key) == CMTV_OK);
  CHECK(bad_key == (int64_t)v.n && !all_ok && out[v.n] == 0 && out[v.n + 1] == 0);
  for (size_t i = 0; i < v.n; i++) CHECK(out[i] == v.go[i]);
  cmtv_batch_reset(b);
  CHECK(cmtv_batch_len(b) == 0);
  cmtv_batch_free(b);
  // verdict cache on, then off
  CHECK(cmtv_verdict_cache(ctx, 64) == CMTV_OK);
  CHECK(verify_eq(ctx, v, CMTV_MODE_GO_STDLIB));
  CHECK(verify_eq(ctx, v, CMTV_MODE_GO_STDLIB));
  CHECK(cmtv_verdict_cache(ctx, 0) == CMTV_OK);
  // registered keys
  cmtv_keyset* ks = nullptr;
  CHECK(cmtv_register_keys(ctx, v.n, v.pk.data(), &ks) == CMTV_OK);
  if (ks) {
    std::vector<uint32_t> idx(v.n);
    for (size_t i = 0; i < v.n; i++) idx[i] = (uint32_t)i;
    std::vector<uint8_t> got(v.n);
    CHECK(cmtv_verify_ed25519_indexed(ctx, ks, v.n, idx.data(), v.sig.data(), v.msg.data(), v.off.data(),
                                      CMTV_MODE_ZIP215, got.data(), nullptr) == CMTV_OK);
    for (size_t i = 0; i < v.n; i++) CHECK(got[i] == v.zip[i]);
    idx[0] = (uint32_t)v.n;  // out of range
    CHECK(cmtv_verify_ed25519_indexed(ctx, ks, v.n, idx.data(), v.sig.data(), v.msg.data(), v.off.data(),
                                      CMTV_MODE_ZIP215, got.data(), nullptr) == CMTV_EINVAL);
    cmtv_keyset_free(ks);
  }
  // concurrent callers on one context
  std::vector<std::thread> th;
  std::vector<int> ok(threads, 1);
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      for (int it = 0; it < 4; it++) ok[t] &= verify_eq(ctx, v, (uint32_t)((t + it) & 1)) ? 1 : 0;
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < threads; t++) CHECK(ok[t]);
  cmtv_stats st{};
  CHECK(cmtv_stats_get(ctx, &st) == CMTV_OK && st.calls > 0 && st.n_devices == 1);
  cmtv_close(ctx);
  // a sharded context over a repeated ordinal (peer-copy gather)
  setenv("CMTV_SHARD_MIN", "64", 1);
  const int32_t devs[3] = {0, 0, 0};
  cmtv_ctx* multi = nullptr;
  CHECK(cmtv_open_devices(&cfg, devs, 3, &multi) == CMTV_OK);
  unsetenv("CMTV_SHARD_MIN");
  if (multi) {
    CHECK(cmtv_device_count(multi) == 3);
    CHECK(verify_eq(multi, v, CMTV_MODE_GO_STDLIB));
    CHECK(verify_eq(multi, v, CMTV_MODE_ZIP215));
    CHECK(cmtv_stats_get(multi, &st) == CMTV_OK && st.sharded_calls >= 2);
    cmtv_close(multi);
  }
}

// A node's goroutines on one context (SURVEY 8b Threading): a blocksync
// caller running pipelined cmtv_verify_commits (CMTV_PIPE_MIN=1 at open, the
// commits' arrays in the context's pinned memory so direct and packed chunks
// both run), a consensus caller running single-commit cmtv_verify_commit, and
// a third thread with host batches -- on a chain signed on the device, with
// a flipped signature every 5th height; every outcome checked.
static void commit_concurrency(int iters) {
  setenv("CMTV_PIPE_MIN", "1", 1);
  setenv("CMTV_PIPE_CHUNK", "512", 1);
  cmtv_ctx* ctx = nullptr;
  cmtv_config cfg{0, CMTV_MODE_GO_STDLIB, 0, 0};
  CHECK(cmtv_open(&cfg, &ctx) == CMTV_OK);
  unsetenv("CMTV_PIPE_MIN");
  unsetenv("CMTV_PIPE_CHUNK");
  if (!ctx) return;
  CHECK(cmtv_keyset_cache(ctx, 2) == CMTV_OK);
  const uint32_t nv = 16, H = 60;
  std::vector<uint8_t> seeds(32 * nv), pk(32 * nv), addrs(20 * nv);
  for (uint32_t i = 0; i < 32 * nv; i++) seeds[i] = (uint8_t)(i * 37 + 11);
  CHECK(cmtv_pubkeys_ed25519(ctx, nv, seeds.data(), pk.data()) == CMTV_OK);
  for (uint32_t i = 0; i < nv; i++) std::memcpy(&addrs[20 * i], &pk[32 * i], 20);
  std::vector<uint32_t> pk_off(nv + 1);
  std::vector<int64_t> power(nv, 10);
  for (uint32_t i = 0; i <= nv; i++) pk_off[i] = 32 * i;
  const cmtv_valset vs{nv, pk.data(), pk_off.data(), power.data(), addrs.data(), nullptr};
  // the arena: flags, seconds, nanos, sig_off, signatures per height
  const size_t per = 8 * ((nv + 1 + 7) / 8 + (nv + 1) + (4 * (nv + 1) + 7) / 8 + (4 * (nv + 1) + 7) / 8) + 64 * nv;
  uint8_t* arena = nullptr;
  CHECK(cmtv_alloc_pinned(ctx, per * H + 4096, reinterpret_cast<void**>(&arena)) == CMTV_OK);
  if (!arena) {
    cmtv_close(ctx);
    return;
  }
  std::vector<uint8_t> bh(32 * H), ph(32 * H);
  std::vector<cmtv_commit> cs(H);
  std::vector<cmtv_block_id> bids(H);
  std::vector<cmtv_valset> vals(H, vs);
  std::vector<int64_t> hs(H);
  const char chain[] = "cmtverify-abicheck";
  size_t at = 0;
  auto carve = [&](size_t bytes) {
    uint8_t* p = arena + at;
    at += (bytes + 7) / 8 * 8;
    return p;
  };
  for (uint32_t h = 0; h < H; h++) {
    for (int k = 0; k < 32; k++) {
      bh[32 * h + k] = (uint8_t)(h * 5 + k);
      ph[32 * h + k] = (uint8_t)(h * 9 + 3 * k);
    }
    bids[h] = cmtv_block_id{&bh[32 * h], 32, 1, &ph[32 * h], 32};
    hs[h] = 100 + h;
    uint8_t* fl = carve(nv + 1);
    auto* se = reinterpret_cast<int64_t*>(carve(8 * (nv + 1)));
    auto* na = reinterpret_cast<int32_t*>(carve(4 * (nv + 1)));
    auto* so = reinterpret_cast<uint32_t*>(carve(4 * (nv + 1)));
    uint8_t* sg = carve(64 * nv);
    std::string msgs;
    std::vector<uint32_t> off{0};
    for (uint32_t i = 0; i < nv; i++) {
      fl[i] = h % 4 == 3 && i == 2 ? 3 : 2;  // a nil vote now and then
      se[i] = 1700000000 + h;
      na[i] = (int32_t)(1000 * i);
      so[i] = 64 * i;
      uint8_t b[256];
      static const cmtv_block_id zero{};
      const int64_t ml = cmtv_vote_sign_bytes(chain, sizeof chain - 1, 2, hs[h], 0, fl[i] == 2 ? &bids[h] : &zero,
                                              se[i], na[i], b, sizeof b);
      msgs.append(reinterpret_cast<const char*>(b), (size_t)ml);
      off.push_back((uint32_t)msgs.size());
    }
    so[nv] = 64 * nv;
    std::vector<uint32_t> kidx(nv);
    for (uint32_t i = 0; i < nv; i++) kidx[i] = i;
    CHECK(cmtv_sign_ed25519(ctx, nv, seeds.data(), kidx.data(), reinterpret_cast<const uint8_t*>(msgs.data()),
                            off.data(), sg) == CMTV_OK);
    if (h % 5 == 1) sg[64 * (h % nv) + 7] ^= 4;  // a wrong signature at index h % nv
    cs[h] = cmtv_commit{hs[h], 0, bids[h], nv, fl, se, na, sg, so, addrs.data()};
  }
  auto expect_ok = [&](uint32_t h, uint32_t kind, int rc, const cmtv_commit_result& r) {
    // VerifyCommitLight stops after floor(2/3 * 160 / 10) + 1 = 11 commit votes
    const uint32_t bad = h % nv;
    const bool flipped = h % 5 == 1;
    // (a nil vote at index 2 every 4th height: skipped by the light loop)
    const bool reached = kind == 0 || (h % 4 == 3 ? bad != 2 && bad < 12 : bad < 11);
    if (flipped && reached) return rc == CMTV_ECOMMIT && r.code == CMTV_COMMIT_ERR_WRONG_SIGNATURE && r.sig_index == (int32_t)bad;
    return rc == CMTV_OK;
  };
  std::vector<int> oks(3, 1);
  std::thread blocksync([&] {
    std::vector<cmtv_commit_result> res(H);
    std::vector<int> rcs(H);
    for (int it = 0; it < iters; it++) {
      const uint32_t kind = (uint32_t)(it & 1);
      if (cmtv_verify_commits(ctx, kind, 0, chain, sizeof chain - 1, H, vals.data(), bids.data(), hs.data(), cs.data(),
                              1, 3, res.data(), rcs.data(), nullptr, 0) != CMTV_OK) {
        oks[0] = 0;
        continue;
      }
      for (uint32_t h = 0; h < H; h++) oks[0] &= expect_ok(h, kind, rcs[h], res[h]) ? 1 : 0;
    }
  });
  std::thread consensus([&] {
    for (int it = 0; it < iters; it++)
      for (uint32_t h = (uint32_t)it % 3; h < H; h += 3) {
        const uint32_t kind = (uint32_t)((it + h) & 1);
        cmtv_commit_result r{};
        const int rc = cmtv_verify_commit(ctx, kind, 0, chain, sizeof chain - 1, &vs, &bids[h], hs[h], &cs[h], 1, 3,
                                          &r, nullptr, 0);
        oks[1] &= expect_ok(h, kind, rc, r) ? 1 : 0;
      }
  });
  std::thread rpc([&] {
    std::vector<uint8_t> m(1, 0), v(nv);
    std::vector<uint32_t> off(nv + 1, 0);
    for (int it = 0; it < 4 * iters; it++) {
      // one height's signatures over empty messages: all invalid
      oks[2] &= cmtv_verify_ed25519(ctx, nv, pk.data(), cs[it % H].sigs, m.data(), off.data(), 0, v.data(), nullptr) ==
                CMTV_OK;
      for (uint32_t i = 0; i < nv; i++) oks[2] &= v[i] == 0;
    }
  });
  blocksync.join();
  consensus.join();
  rpc.join();
  CHECK(oks[0] && oks[1] && oks[2]);
  cmtv_stats st{};
  CHECK(cmtv_stats_get(ctx, &st) == CMTV_OK && st.direct_chunks > 0);
  CHECK(cmtv_free_pinned(ctx, arena) == CMTV_OK);
  cmtv_close(ctx);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  Vecs v;
  if (!load(argv[1], v)) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  const int threads = argc > 2 ? std::atoi(argv[2]) : 4;
  device_free_checks();
  cmtv_ctx* probe = nullptr;
  const int rc = cmtv_open(nullptr, &probe);
  if (rc == CMTV_ENODEV) {
    std::printf("no device: device-free checks only\n");
  } else {
    CHECK(rc == CMTV_OK);
    cmtv_close(probe);
    device_checks(v, threads);
    commit_concurrency(4);
  }
  std::printf("abicheck: %zu vectors, %d failures\n", v.n, fails);
  std::fflush(stdout);
  // Every context is closed by now. With a device, skip the static
  // destructors: the HIP runtime's run after the sanitizer's device
  // allocator considers the device runtime unloaded, and a device chunk it
  // recycles from its quarantine during that teardown trips a sanitizer
  // CHECK (round 6: AddressSanitizer sanitizer_allocator_device.h:125 from
  // __cxa_finalize of libamdhip64, after the checks had passed). Leak
  // detection is off for this binary (tests/test_sanitizers.py).
  if (rc != CMTV_ENODEV) std::_Exit(fails ? 1 : 0);
  return fails ? 1 : 0;
}
