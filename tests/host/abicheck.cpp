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
  }
  std::printf("abicheck: %zu vectors, %d failures\n", v.n, fails);
  return fails ? 1 : 0;
}
