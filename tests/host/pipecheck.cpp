// pipecheck.cpp -- CPU check of cmtv_verify_commits' host logic: the commit
// layer (commit.cpp) and the chunked cross-height pipeline (pipeline.cpp)
// linked against tests/host/fake_runtime.cpp, whose "device" verifies with
// the C restatement of Go 1.19 ed25519.Verify (oracle/cmtv_oracle.c).
//
// A chain of commits with assorted faults over four validator sets is
// verified three ways and must agree on every commit:
//   ref       the reference loops, written out here from
//             types/validator_set.go:667-826 (one VerifySignature per
//             signature the loop reaches: crypto/ed25519/ed25519.go:148-155)
//   one       cmtv_verify_commits' one-batch path (pipeline off)
//   pipe      the pipeline over many configurations: chunk sizes down to a
//             few signatures, 2-4 slots, 1-8 host threads, 1-3 devices,
//             registered keys on and off, a device failing mid-call
// ref vs one/pipe: return code, error code, index, got/needed; one vs pipe:
// the whole result struct and error string, byte for byte.
// Usage: pipecheck [n_heights]; exit 0 = all agree.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cmtverify.h"
#include "../../cometbft_amd/csrc/commit_internal.h"

extern "C" {
int oracle_verify_one(const uint8_t* pk, const uint8_t* msg, size_t mlen, const uint8_t* sig, int mode);
void oracle_pubkey_from_seed(const uint8_t seed[32], uint8_t pk[32]);
void oracle_sign(const uint8_t seed[32], const uint8_t* msg, size_t mlen, uint8_t sig[64]);
cmtv_ctx* fake_open(size_t n_devs, unsigned threads, size_t pipe_min, size_t chunk, int slots, bool pipe_on,
                    size_t keyset_cap, long fail_dev);
void fake_counts(cmtv_ctx* c, uint64_t* out);
void fake_set_ext_retire(cmtv_ctx* c, long dev);
void fake_set_direct(cmtv_ctx* c, bool on);
void fake_set_span(cmtv_ctx* c, uint64_t factor, uint64_t slack);
void fake_set_keyset_fail(cmtv_ctx* c, bool on);
void fake_close(cmtv_ctx* c);
}

namespace {

const char kChain[] = "cmtverify-pipecheck";

struct VSet {
  std::vector<uint8_t> seeds, pk, addrs;
  std::vector<uint32_t> pk_off;
  std::vector<int64_t> power, prio;
  cmtv_valset vs{};
  void finish() {
    vs.n_vals = (uint32_t)power.size();
    vs.pubkeys = pk.data();
    vs.pk_off = pk_off.data();
    vs.voting_power = power.data();
    vs.addrs = addrs.data();
    vs.proposer_priority = prio.data();
  }
};

void make_set(VSet& v, uint32_t n, uint32_t seed0, int bad_key = -1) {
  v.pk_off.push_back(0);
  for (uint32_t i = 0; i < n; i++) {
    uint8_t seed[32] = {0}, pk[32];
    std::memcpy(seed, &seed0, 4);
    std::memcpy(seed + 4, &i, 4);
    seed[31] = 0x5A;
    oracle_pubkey_from_seed(seed, pk);
    v.seeds.insert(v.seeds.end(), seed, seed + 32);
    const uint32_t len = (int)i == bad_key ? 31 : 32;
    v.pk.insert(v.pk.end(), pk, pk + len);
    v.pk_off.push_back(v.pk_off.back() + len);
    v.addrs.insert(v.addrs.end(), pk, pk + 20);  // unique per key (the harness needs no SHA-256)
    v.power.push_back(10 + (i % 3));
    v.prio.push_back((int64_t)i - 5);
  }
  v.finish();  // pointers into v's own vectors: v is built in place, never copied
}

struct CommitData {
  std::vector<uint8_t> flags, sigs, vaddr, bh, ph;
  std::vector<int64_t> sec;
  std::vector<int32_t> nanos;
  std::vector<uint32_t> sig_off;
  cmtv_commit c{};
  cmtv_block_id want{};  // the block ID the caller expects
  int64_t height = 0;    // the height the caller expects
  const VSet* set = nullptr;
};

std::vector<uint8_t> sign_bytes(const cmtv_commit& c, uint32_t idx) {
  static const cmtv_block_id empty{};
  const cmtv_block_id* b = c.flags[idx] == 2 ? &c.block_id : &empty;
  uint8_t buf[512];
  const int64_t n = cmtv_vote_sign_bytes(kChain, sizeof kChain - 1, 2, c.height, c.round, b, c.ts_seconds[idx],
                                         c.ts_nanos[idx], buf, sizeof buf);
  return std::vector<uint8_t>(buf, buf + n);
}

void make_commit(CommitData& d, const VSet& s, int64_t h) {
  const uint32_t n = s.vs.n_vals;
  d.set = &s;
  d.flags.assign(n + 1, 2);
  for (uint32_t i = 0; i < n; i++) {
    if (h % 7 == 0 && i % 4 == 0) d.flags[i] = 3;   // nil votes
    if (h % 11 == 0 && i < 8) d.flags[i] = 1;       // absent
    if (h % 43 == 0 && i < n / 2) d.flags[i] = 1;   // too few signatures
  }
  d.bh.resize(32);
  d.ph.resize(32);
  for (int k = 0; k < 32; k++) {
    d.bh[k] = (uint8_t)(h * 31 + k);
    d.ph[k] = (uint8_t)(h * 17 + 3 * k);
  }
  d.sec.resize(n);
  d.nanos.resize(n);
  d.vaddr.resize(20 * (size_t)n + 1);
  for (uint32_t i = 0; i < n; i++) {
    d.sec[i] = 1672531200 + h;
    d.nanos[i] = (int32_t)(i * 1000 + (h % 5 == 0 ? 999999 : 0));
    if (h % 9 == 0 && i == 3) d.nanos[i] = 0;  // a zero field is omitted
    std::memcpy(&d.vaddr[20 * (size_t)i], &s.addrs[20 * (size_t)i], 20);
  }
  d.c.height = h;
  d.c.round = h % 6 == 0 ? 2 : 0;
  d.c.block_id = cmtv_block_id{d.bh.data(), 32, 1, d.ph.data(), 32};
  d.c.n_sigs = n;
  d.c.flags = d.flags.data();
  d.c.ts_seconds = d.sec.data();
  d.c.ts_nanos = d.nanos.data();
  // signatures (absent: empty), then the faults
  std::vector<std::vector<uint8_t>> sg(n);
  for (uint32_t i = 0; i < n; i++) {
    if (d.flags[i] == 1) continue;
    sg[i].resize(64);
    const auto m = sign_bytes(d.c, i);
    oracle_sign(&s.seeds[32 * (size_t)i], m.data(), m.size(), sg[i].data());
  }
  auto flip = [&](uint32_t i, int byte, int bit) {
    if (i < n && sg[i].size() == 64) sg[i][byte] ^= (uint8_t)bit;
  };
  if (h % 13 == 0) flip(2, 10, 1);
  if (h % 17 == 0) flip(n - 1, 40, 4);
  if (h % 19 == 0 && sg[5].size()) sg[5].pop_back();           // 63 bytes
  if (h % 47 == 0 && sg[9].size()) sg[9].push_back(0);         // 65 bytes
  if (h % 29 == 0) d.flags[10] = 7;                            // unknown BlockIDFlag
  if (h % 31 == 0) std::memcpy(&d.vaddr[20 * 6], &d.vaddr[20 * 4], 20);  // double vote
  if (h % 37 == 0) std::memset(&d.vaddr[20 * 7], 0, 20);      // unknown validator
  if (h % 53 == 0) flip(1, 0, 0x80);                           // R' mismatch in the first byte
  if (h % 59 == 0 && sg[12].size()) sg[12][63] |= 0xE0;        // sig[63] high bits
  d.sig_off.assign(1, 0);
  for (uint32_t i = 0; i < n; i++) {
    d.sigs.insert(d.sigs.end(), sg[i].begin(), sg[i].end());
    d.sig_off.push_back((uint32_t)d.sigs.size());
  }
  d.sigs.push_back(0);
  d.c.sigs = d.sigs.data();
  d.c.sig_off = d.sig_off.data();
  d.c.val_addrs = d.vaddr.data();
  d.height = h % 23 == 0 ? h + 1 : h;
  d.want = d.c.block_id;
  if (h % 41 == 0) d.want.psh_total = 2;  // wrong block ID
}

// ---------------------------------------------------------------- reference

struct Outcome {
  int rc = 0;  // CMTV_OK or CMTV_ECOMMIT
  int32_t code = 0, index = -1;
  int64_t got = 0, needed = 0;
};

std::map<std::string, bool> g_memo;

// PubKey.VerifySignature (crypto/ed25519/ed25519.go:148-155): false for a
// signature that is not 64 bytes; Go's ed25519.Verify panics on a key that
// is not 32 bytes (returned here as panicked)
bool verify_signature(const VSet& s, uint32_t vi, const std::vector<uint8_t>& msg, const uint8_t* sig,
                      uint32_t sig_len, int mode, bool* panicked) {
  *panicked = false;
  if (sig_len != 64) return false;
  if (s.pk_off[vi + 1] - s.pk_off[vi] != 32) {
    *panicked = true;
    return false;
  }
  const uint8_t* pk = &s.pk[s.pk_off[vi]];
  std::string k(1, (char)mode);
  k.append((const char*)pk, 32).append((const char*)sig, 64).append((const char*)msg.data(), msg.size());
  auto it = g_memo.find(k);
  if (it != g_memo.end()) return it->second;
  const bool v = oracle_verify_one(pk, msg.data(), msg.size(), sig, mode) != 0;
  g_memo.emplace(k, v);
  return v;
}

Outcome fail(int32_t code, int32_t idx) {
  Outcome o;
  o.rc = CMTV_ECOMMIT;
  o.code = code;
  o.index = idx;
  return o;
}

bool bid_equal(const cmtv_block_id& a, const cmtv_block_id& b) {
  return a.hash_len == b.hash_len && !std::memcmp(a.hash, b.hash, a.hash_len) && a.psh_total == b.psh_total &&
         a.psh_hash_len == b.psh_hash_len && !std::memcmp(a.psh_hash, b.psh_hash, a.psh_hash_len);
}

// types/validator_set.go:667-714 (kind 0), 722-765 (kind 1), 775-826 (kind 2)
Outcome reference(uint32_t kind, int mode, const VSet& vals, const CommitData& d, uint64_t tn, uint64_t td) {
  const cmtv_commit& c = d.c;
  int64_t total = 0;
  for (auto p : vals.power) total += p;
  int64_t needed;
  if (kind == 2) {
    if (td == 0) return fail(CMTV_COMMIT_ERR_TRUST_LEVEL, -1);
    needed = total * (int64_t)tn / (int64_t)td;  // no overflow at these sizes
  } else {
    if (vals.vs.n_vals != c.n_sigs) return fail(CMTV_COMMIT_ERR_SET_SIZE, -1);
    if (d.height != c.height) return fail(CMTV_COMMIT_ERR_HEIGHT, -1);
    if (!bid_equal(d.want, c.block_id)) return fail(CMTV_COMMIT_ERR_BLOCK_ID, -1);
    needed = total * 2 / 3;
  }
  int64_t tally = 0;
  std::map<uint32_t, uint32_t> seen;
  for (uint32_t idx = 0; idx < c.n_sigs; idx++) {
    const uint8_t f = c.flags[idx];
    uint32_t vi = idx;
    if (kind == 0) {
      if (f == 1) continue;
      if (f != 2 && f != 3) return fail(CMTV_COMMIT_PANIC_UNKNOWN_FLAG, (int32_t)idx);  // VoteSignBytes
    } else {
      if (f != 2) continue;
      if (kind == 2) {
        int64_t found = -1;
        for (uint32_t j = 0; j < vals.vs.n_vals && found < 0; j++)
          if (!std::memcmp(&vals.addrs[20 * (size_t)j], c.val_addrs + 20 * (size_t)idx, 20)) found = j;
        if (found < 0) continue;
        vi = (uint32_t)found;
        auto it = seen.find(vi);
        if (it != seen.end()) {
          Outcome o = fail(CMTV_COMMIT_ERR_DOUBLE_VOTE, (int32_t)idx);
          o.got = it->second;
          o.needed = vi;
          return o;
        }
        seen[vi] = idx;
      }
    }
    bool panicked = false;
    const bool ok = verify_signature(vals, vi, sign_bytes(c, idx), c.sigs + c.sig_off[idx],
                                     c.sig_off[idx + 1] - c.sig_off[idx], mode, &panicked);
    if (panicked) return fail(CMTV_COMMIT_PANIC_BAD_PUBKEY, (int32_t)idx);
    if (!ok) return fail(CMTV_COMMIT_ERR_WRONG_SIGNATURE, (int32_t)idx);
    if (kind == 0) {
      if (f == 2) tally += vals.power[vi];
    } else {
      tally += vals.power[vi];
      if (tally > needed) return Outcome();
    }
  }
  if (kind == 0 && tally > needed) return Outcome();
  Outcome o = fail(CMTV_COMMIT_ERR_NOT_ENOUGH_POWER, -1);
  o.got = tally;
  o.needed = needed;
  return o;
}

// ---------------------------------------------------------------- library runs

struct Run {
  std::vector<int> rcs;
  std::vector<cmtv_commit_result> res;
  std::vector<char> msgs;
};

constexpr size_t kCap = 1024;

// Where the caller's commit arrays live (cmtv_alloc_pinned: the direct
// chunks' DMA source, pipeline.cpp):
//   kHeap         the CommitData vectors themselves (packed chunks only)
//   kInterleaved  one pinned block, per commit flags | secs | nanos | sig_off |
//                 sigs (the Go shim's arena)
//   kClasses      one pinned block, all flags, then all secs, nanos, sigs
//   kMisaligned   interleaved, every third commit's signatures 4 bytes off
//                 (not direct: the kernel loads 8-byte words)
enum Layout { kHeap, kInterleaved, kClassArrays, kMisaligned };

std::vector<cmtv_commit> place(cmtv_ctx* ctx, const std::vector<CommitData>& chain, Layout lay) {
  std::vector<cmtv_commit> cs;
  for (auto& d : chain) cs.push_back(d.c);
  if (lay == kHeap) return cs;
  size_t bytes = 4096;
  for (auto& d : chain) bytes += 64 + d.flags.size() + 8 * d.sec.size() + 4 * d.nanos.size() + 4 * d.sig_off.size() +
                                 d.sigs.size() + 64;
  uint8_t* blk = nullptr;
  if (cmtv_alloc_pinned(ctx, bytes, reinterpret_cast<void**>(&blk)) != CMTV_OK) {
    std::fprintf(stderr, "cmtv_alloc_pinned failed\n");
    std::exit(2);
  }
  size_t at = 0;
  auto put = [&](const void* src, size_t len, size_t align, size_t skew = 0) {
    at = (at + align - 1) / align * align + skew;
    std::memcpy(blk + at, src, len);
    const uint8_t* p = blk + at;
    at += len;
    return p;
  };
  for (int pass = 0; pass < (lay == kClassArrays ? 4 : 1); pass++)
    for (size_t i = 0; i < chain.size(); i++) {
      const CommitData& d = chain[i];
      cmtv_commit& c = cs[i];
      const size_t n = d.sec.size();
      auto cls = [&](int k) { return lay != kClassArrays || pass == k; };
      if (cls(0)) c.flags = put(d.flags.data(), d.flags.size(), 1);
      if (cls(1)) c.ts_seconds = reinterpret_cast<const int64_t*>(put(d.sec.data(), 8 * n, 8));
      if (cls(2)) c.ts_nanos = reinterpret_cast<const int32_t*>(put(d.nanos.data(), 4 * n, 4));
      if (cls(3)) {
        c.sig_off = reinterpret_cast<const uint32_t*>(put(d.sig_off.data(), 4 * d.sig_off.size(), 4));
        c.sigs = put(d.sigs.data(), d.sigs.size(), 8, lay == kMisaligned && i % 3 == 0 ? 4 : 0);
      }
    }
  return cs;
}

Run run(cmtv_ctx* ctx, uint32_t kind, uint32_t mode, const std::vector<CommitData>& chain,
        const std::vector<const VSet*>& vals_of, Layout lay = kHeap) {
  const size_t n = chain.size();
  std::vector<cmtv_valset> vs(n);
  std::vector<cmtv_block_id> bids(n);
  std::vector<int64_t> hs(n);
  const std::vector<cmtv_commit> cs = place(ctx, chain, lay);
  for (size_t i = 0; i < n; i++) {
    vs[i] = vals_of[i]->vs;
    bids[i] = chain[i].want;
    hs[i] = chain[i].height;
  }
  Run r;
  r.rcs.assign(n, 99);
  r.res.assign(n, cmtv_commit_result{});
  r.msgs.assign(n * kCap, 0);
  const int rc = cmtv_verify_commits(ctx, kind, mode, kChain, sizeof kChain - 1, n, vs.data(),
                                     kind == 2 ? nullptr : bids.data(), hs.data(), cs.data(), 1, 3, r.res.data(),
                                     r.rcs.data(), r.msgs.data(), kCap);
  if (rc != CMTV_OK) {
    std::fprintf(stderr, "cmtv_verify_commits: %d\n", rc);
    std::exit(2);
  }
  return r;
}

int g_fail = 0;

void expect_same_as_ref(const char* what, uint32_t kind, const Run& r, const std::vector<Outcome>& ref) {
  for (size_t i = 0; i < ref.size(); i++) {
    const Outcome& o = ref[i];
    const cmtv_commit_result& x = r.res[i];
    bool ok = r.rcs[i] == o.rc;
    if (ok && o.rc != CMTV_OK) {
      ok = x.code == o.code && x.sig_index == o.index;
      if (o.code == CMTV_COMMIT_ERR_NOT_ENOUGH_POWER || o.code == CMTV_COMMIT_ERR_DOUBLE_VOTE)
        ok = ok && x.got == o.got && x.needed == o.needed;
    }
    if (!ok) {
      if (g_fail++ < 20)
        std::fprintf(stderr, "%s kind %u commit %zu: rc %d code %d idx %d got %lld needed %lld; ref rc %d code %d idx %d "
                     "got %lld needed %lld: %s\n", what, kind, i, r.rcs[i], x.code, x.sig_index, (long long)x.got,
                     (long long)x.needed, o.rc, o.code, o.index, (long long)o.got, (long long)o.needed,
                     &r.msgs[i * kCap]);
    }
  }
}

void expect_same(const char* what, const Run& a, const Run& b) {
  if (a.rcs != b.rcs || std::memcmp(a.res.data(), b.res.data(), a.res.size() * sizeof(cmtv_commit_result)) ||
      a.msgs != b.msgs) {
    for (size_t i = 0; i < a.rcs.size(); i++)
      if (a.rcs[i] != b.rcs[i] || std::memcmp(&a.res[i], &b.res[i], sizeof(cmtv_commit_result)) ||
          std::memcmp(&a.msgs[i * kCap], &b.msgs[i * kCap], kCap)) {
        if (g_fail++ < 20)
          std::fprintf(stderr, "%s: commit %zu differs from the one-batch path: rc %d vs %d, '%s' vs '%s'\n", what, i,
                       b.rcs[i], a.rcs[i], &b.msgs[i * kCap], &a.msgs[i * kCap]);
        break;
      }
  }
}

}  // namespace

// Concurrency (pipecheck <heights> race; built with -fsanitize=thread by
// tests/test_pipeline_cpu.py): callers share one context as a node's
// goroutines do (SURVEY 8b Threading) -- a blocksync goroutine running
// pipelined cmtv_verify_commits (direct and packed chunks over two fake
// devices, host worker pool), a consensus goroutine running single-commit
// cmtv_verify_commit calls, and an RPC-like reader of the context's pinned
// blocks allocating and freeing its own -- each checking every outcome
// against the reference loops.
int race(const std::vector<CommitData>& chain, const std::vector<const VSet*>& vals_of, int iters) {
  std::vector<Outcome> ref[2];
  for (uint32_t kind = 0; kind < 2; kind++)
    for (size_t i = 0; i < chain.size(); i++) ref[kind].push_back(reference(kind, 0, *vals_of[i], chain[i], 1, 3));
  cmtv_ctx* ctx = fake_open(2, 4, 1, 64, 2, true, 4, -1);
  std::atomic<int> bad{0};
  std::thread pipe([&] {
    for (int it = 0; it < iters; it++) {
      const uint32_t kind = (uint32_t)(it & 1);
      const Run r = run(ctx, kind, 0, chain, vals_of, it % 3 == 2 ? kHeap : kInterleaved);
      for (size_t i = 0; i < chain.size(); i++)
        if (r.rcs[i] != ref[kind][i].rc || (r.rcs[i] && r.res[i].code != ref[kind][i].code)) bad++;
    }
  });
  std::thread single([&] {
    for (int it = 0; it < iters; it++)
      for (size_t i = 0; i < chain.size(); i += 7) {
        const uint32_t kind = (uint32_t)((it + i) & 1);
        cmtv_commit_result res{};
        char msg[256];
        const int rc = cmtv_verify_commit(ctx, kind, 0, kChain, sizeof kChain - 1, &vals_of[i]->vs, &chain[i].want,
                                          chain[i].height, &chain[i].c, 1, 3, &res, msg, sizeof msg);
        if (rc != ref[kind][i].rc || (rc && res.code != ref[kind][i].code)) bad++;
      }
  });
  std::thread other([&] {
    for (int it = 0; it < 50 * iters; it++) {
      void* p = nullptr;
      if (cmtv_alloc_pinned(ctx, 4096 + 64 * (size_t)it, &p) != CMTV_OK || cmtv_free_pinned(ctx, p) != CMTV_OK) bad++;
    }
  });
  pipe.join();
  single.join();
  other.join();
  uint64_t cnt[8];
  fake_counts(ctx, cnt);
  fake_close(ctx);
  if (!cnt[5]) {
    std::fprintf(stderr, "race: no direct chunk ran\n");
    bad++;
  }
  std::printf("race: %d iterations, %d mismatches\n", iters, bad.load());
  return bad ? 1 : 0;
}

// commit_template_lens (the pipeline's plan) == put_commit_template's
// lengths (what the pack writes) over heights, rounds, block IDs and chain ids
int check_template_lens() {
  int bad = 0;
  uint8_t h1[300], h2[300];
  for (int i = 0; i < 300; i++) h1[i] = h2[i] = (uint8_t)i;
  const int64_t heights[] = {0, 1, -1, 127, 1ll << 40, INT64_MIN};
  const int32_t rounds[] = {0, 1, -5, INT32_MAX};
  const uint32_t lens[] = {0, 1, 32, 127, 128, 200};
  const uint32_t totals[] = {0, 1, 127, 128, 1u << 31};
  const size_t chains[] = {0, 1, 15, 50, 127, 128, 200};
  static char chain[256];
  for (int64_t h : heights)
    for (int32_t r : rounds)
      for (uint32_t hl : lens)
        for (uint32_t pl : lens)
          for (uint32_t tot : totals)
            for (size_t cl : chains) {
              cmtv_commit c{};
              c.height = h;
              c.round = r;
              c.block_id = cmtv_block_id{h1, hl, tot, h2, pl};
              cmtv::SbTemplate t{};
              const size_t n = cmtv::put_commit_template(nullptr, 0, chain, cl, &c, &t);
              uint32_t a, b, p;
              const size_t m = cmtv::commit_template_lens(cl, &c, &a, &b, &p);
              if (n != m || a != t.pre_commit_len || b != t.pre_nil_len || p != t.post_len) bad++;
            }
  if (bad) std::fprintf(stderr, "commit_template_lens differs in %d cases\n", bad);
  return bad;
}

// Single-commit cmtv_verify_commit with the keyset cache, the speculative
// path on (CMTV_SPEC_MIN=1): every commit twice (the first call registers its
// set, the second launches on the guessed set before checking anything per
// signature), against the reference loops; then a set whose key bytes change
// in place between calls (the guess must be refuted by the byte compare).
int check_single(const std::vector<CommitData>& chain, const std::vector<const VSet*>& vals_of) {
  int bad = 0;
  uint64_t spec = 0, spec_ok = 0, cnt[8];
  for (uint32_t kind = 0; kind < 3; kind++) {
    cmtv_ctx* ctx = fake_open(1, 2, 1, 1u << 20, 3, true, 4, -1);
    for (int pass = 0; pass < 2; pass++)
      for (size_t i = 0; i < chain.size(); i++) {
        const Outcome o = reference(kind, 0, *vals_of[i], chain[i], 1, 3);
        cmtv_commit_result res{};
        char msg[512];
        const int rc = cmtv_verify_commit(ctx, kind, 0, kChain, sizeof kChain - 1, &vals_of[i]->vs, &chain[i].want,
                                          chain[i].height, &chain[i].c, 1, 3, &res, msg, sizeof msg);
        if (rc != o.rc || (rc != CMTV_OK && (res.code != o.code || res.sig_index != o.index))) {
          if (bad++ < 10)
            std::fprintf(stderr, "single kind %u pass %d commit %zu: rc %d code %d idx %d, ref rc %d code %d idx %d\n",
                         kind, pass, i, rc, res.code, res.sig_index, o.rc, o.code, o.index);
        }
      }
    fake_counts(ctx, cnt);
    spec += cnt[6];
    spec_ok += cnt[7];
    fake_close(ctx);
  }
  // speculation ran (VerifyCommit / Light), held where the commit is clean and
  // was refuted where it is not (faulty heights)
  if (!spec || spec_ok == spec || !spec_ok) {
    std::fprintf(stderr, "single: %llu speculative launches, %llu held\n", (unsigned long long)spec,
                 (unsigned long long)spec_ok);
    bad++;
  }
  // the keys of set A rewritten in place with another set's key at index 3
  const CommitData& d = chain[0];
  const VSet& A = *d.set;
  VSet A2 = A;  // vectors copied; pointers re-aimed below
  std::vector<uint8_t> keys(A.pk);
  A2.vs.pubkeys = keys.data();
  A2.vs.pk_off = A.pk_off.data();
  A2.vs.voting_power = A.power.data();
  A2.vs.addrs = A.addrs.data();
  A2.vs.proposer_priority = A.prio.data();
  cmtv_ctx* ctx = fake_open(1, 1, 1, 1u << 20, 3, true, 4, -1);
  for (int round = 0; round < 3; round++) {
    if (round == 2) std::memcpy(&keys[32 * 3], &keys[32 * 4], 32);  // same pointer, other bytes
    std::memcpy(A2.pk.data(), keys.data(), keys.size());
    A2.vs.pubkeys = keys.data();
    const Outcome o = reference(0, 0, A2, d, 1, 3);
    cmtv_commit_result res{};
    const int rc = cmtv_verify_commit(ctx, 0, 0, kChain, sizeof kChain - 1, &A2.vs, &d.want, d.height, &d.c, 1, 3,
                                      &res, nullptr, 0);
    if (rc != o.rc || (rc != CMTV_OK && (res.code != o.code || res.sig_index != o.index))) {
      bad++;
      std::fprintf(stderr, "single, keys rewritten (round %d): rc %d code %d idx %d, ref rc %d idx %d\n", round, rc,
                   res.code, res.sig_index, o.rc, o.index);
    }
    if (round == 2 && (rc != CMTV_ECOMMIT || res.sig_index != 3)) bad++;  // key 3 changed: its signature fails
  }
  fake_counts(ctx, cnt);
  if (cnt[6] != 2 || cnt[7] != 1) {  // rounds 1 and 2 speculate; round 2's guess is refuted
    std::fprintf(stderr, "single, keys rewritten: %llu speculative launches, %llu held\n",
                 (unsigned long long)cnt[6], (unsigned long long)cnt[7]);
    bad++;
  }
  fake_close(ctx);
  std::printf("single: %zu commits x 3 kinds x 2, %d mismatches\n", chain.size(), bad);
  return bad;
}

int main(int argc, char** argv) {
  setenv("CMTV_SPEC_MIN", "1", 1);  // the speculative single-commit path at any size
  const int64_t heights = argc > 1 ? std::atoll(argv[1]) : 240;
  if (check_template_lens()) return 1;
  const bool race_mode = argc > 2 && std::strcmp(argv[2], "race") == 0;
  const uint32_t nv = 24;
  VSet A, B, C, Bad;
  make_set(A, nv, 1);
  make_set(B, nv, 2);
  make_set(C, nv - 6, 3);
  make_set(Bad, nv, 4, 15);
  std::vector<CommitData> chain((size_t)heights);
  std::vector<const VSet*> vals_of;
  for (int64_t h = 1; h <= heights; h++) {
    const int64_t q = (h - 1) * 10 / heights;  // A A A B B B C C Bad A
    const VSet& s = q < 3 || q == 9 ? A : q < 6 ? B : q < 8 ? C : Bad;
    make_commit(chain[(size_t)h - 1], s, h);
    // a bad-key commit whose signature at the bad key is malformed: false
    // before the key-length panic (ed25519.go:150)
    vals_of.push_back(&s);
  }
  for (auto& d : chain)
    if (d.set == &Bad && d.c.height % 5 == 0 && d.sig_off[16] - d.sig_off[15] == 64) {
      // cut signature 15 (the 31-byte key's) to 63 bytes
      d.sigs.erase(d.sigs.begin() + d.sig_off[15] + 63);
      for (size_t i = 16; i < d.sig_off.size(); i++) d.sig_off[i]--;
      d.c.sigs = d.sigs.data();
      d.c.sig_off = d.sig_off.data();
    }
  if (race_mode) return race(chain, vals_of, 6);
  if (check_single(chain, vals_of)) return 1;
  struct Cfg {
    const char* name;
    size_t devs;
    unsigned threads;
    size_t chunk;
    int slots;
    size_t keys;
    long fail_dev;
    long ext_retire = -1;  // retired by "another call" while a chunk is in flight
    Layout lay = kHeap;
    bool direct = true;       // CMTV_PIPE_DIRECT
    bool keyset_fail = false;
    bool tight_spans = false;  // span cap = the plans' bytes: chunks re-cut commit by commit
  };
  const Cfg cfgs[] = {
      {"pipe chunk 1000", 1, 4, 1000, 3, 0, -1},   {"pipe chunk 7", 1, 3, 7, 2, 0, -1},
      {"pipe keyed 64", 1, 8, 64, 2, 4, -1},       {"pipe keyed 1 thread", 1, 1, 200, 3, 4, -1},
      {"pipe 3 devs keyed", 3, 4, 50, 4, 1, -1},   {"pipe 3 devs fail", 3, 2, 80, 2, 4, 1},
      {"pipe keyed cap 1", 2, 5, 30, 3, 1, -1},    {"pipe 2 devs retired elsewhere", 2, 3, 40, 2, 4, -1, 1},
      {"direct interleaved", 1, 4, 100, 3, 4, -1, -1, kInterleaved},
      {"direct classes 2 devs", 2, 4, 64, 2, 4, -1, -1, kClassArrays},
      {"direct misaligned", 1, 3, 50, 2, 4, -1, -1, kMisaligned},
      {"direct 3 devs fail", 3, 2, 80, 2, 4, 1, -1, kInterleaved},
      {"direct big chunks", 2, 8, 4000, 3, 1, -1, -1, kClassArrays},
      {"direct off, pinned", 1, 4, 100, 3, 4, -1, -1, kInterleaved, false},
      {"direct, keys unregistered", 1, 4, 100, 3, 4, -1, -1, kInterleaved, true, true},
      {"direct, tight spans", 2, 4, 100, 3, 4, -1, -1, kInterleaved, true, false, true},
  };
  size_t checked = 0;
  for (uint32_t kind = 0; kind < 3; kind++) {
    for (int mode = 0; mode < 2; mode++) {
      if (kind && mode) continue;  // modes differ only below the replay; both checked on kind 0
      std::vector<Outcome> ref;
      for (size_t i = 0; i < chain.size(); i++) ref.push_back(reference(kind, mode, *vals_of[i], chain[i], 1, 3));
      cmtv_ctx* one = fake_open(1, 1, 1, 1u << 20, 3, false, 0, -1);
      const Run base = run(one, kind, mode, chain, vals_of);
      fake_close(one);
      expect_same_as_ref("one-batch", kind, base, ref);
      cmtv_ctx* onek = fake_open(1, 1, 1, 1u << 20, 3, false, 4, -1);
      expect_same("one-batch keyed", base, run(onek, kind, mode, chain, vals_of));
      fake_close(onek);
      for (const Cfg& c : cfgs) {
        cmtv_ctx* ctx = fake_open(c.devs, c.threads, 1, c.chunk, c.slots, true, c.keys, c.fail_dev);
        fake_set_ext_retire(ctx, c.ext_retire);
        fake_set_direct(ctx, c.direct);
        fake_set_keyset_fail(ctx, c.keyset_fail);
        if (c.tight_spans) fake_set_span(ctx, 1, 0);
        const Run r = run(ctx, kind, mode, chain, vals_of, c.lay);
        uint64_t cnt[8];
        fake_counts(ctx, cnt);
        fake_close(ctx);
        expect_same(c.name, base, r);
        expect_same_as_ref(c.name, kind, r, ref);
        if ((c.fail_dev >= 0 || c.ext_retire >= 0) && cnt[3] != 1) {
          std::fprintf(stderr, "%s: expected one device retired, got %llu\n", c.name, (unsigned long long)cnt[3]);
          g_fail++;
        }
        // direct chunks exactly where they can run (not LightTrusting: its
        // plan maps through addresses)
        const bool want_direct = c.lay != kHeap && c.direct && !c.keyset_fail && c.keys && kind != 2;
        if (want_direct != (cnt[5] > 0)) {
          std::fprintf(stderr, "%s kind %u: %llu direct chunks\n", c.name, kind, (unsigned long long)cnt[5]);
          g_fail++;
        }
        if (c.keys && !c.keyset_fail && !cnt[4]) {
          std::fprintf(stderr, "%s: no chunk used registered keys\n", c.name);
          g_fail++;
        }
        checked++;
      }
      size_t errs = 0;
      for (auto& o : ref) errs += o.rc != CMTV_OK;
      std::printf("kind %u mode %d: %zu commits (%zu with errors) agree across %zu pipeline configs\n", kind, mode,
                  ref.size(), errs, sizeof cfgs / sizeof cfgs[0]);
    }
  }
  if (g_fail) {
    std::fprintf(stderr, "pipecheck: %d mismatches\n", g_fail);
    return 1;
  }
  std::printf("pipecheck ok (%zu runs)\n", checked);
  return 0;
}
