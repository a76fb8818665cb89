// fake_runtime.cpp -- test double of the device half of libcmtverify
// (runtime_internal.h) for tests/host/pipecheck.cpp: the commit layer
// (commit.cpp) and the cross-height pipeline (pipeline.cpp) are linked
// unchanged against it and run on the CPU, so their host logic -- plan,
// pinned-staging layout, chunking, replay, retries -- is checked without a
// GPU and under AddressSanitizer.
//
// The "device" decodes a chunk's staging exactly as the kernels read it
// (keys or key indices, signatures, message offsets, per-commit templates
// written out with signbytes.h sb_write, which must land on the host's
// offsets) and verifies each signature with the C restatement of Go 1.19
// ed25519.Verify (oracle/cmtv_oracle.c). It does so lazily, when the chunk is
// waited for, so a host that rewrote a slot's staging while its chunk was in
// flight reads back wrong verdicts. Test infrastructure only.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../cometbft_amd/csrc/commit_internal.h"
#include "../../cometbft_amd/csrc/host_pool.h"
#include "../../cometbft_amd/csrc/runtime_internal.h"
#include "../../cometbft_amd/csrc/signbytes.h"

extern "C" int oracle_verify_one(const uint8_t* pk, const uint8_t* msg, size_t mlen, const uint8_t* sig, int mode);

struct FakeSlot {
  std::vector<uint8_t> h_in;
  std::vector<uint64_t> bm;
  cmtv::BulkLayout L;
  const cmtv_keyset* ks = nullptr;
  uint32_t mode = 0;
  bool pending = false;
  uint64_t gathered_bytes = 0;  // a direct chunk's message bytes (bulk_gather)
};

struct cmtv_keyset {
  size_t n = 0;
  std::vector<uint8_t> pk;
  int pins = 0;
};

struct cmtv_ctx {
  std::mutex mu, bulk_mu;
  std::unique_ptr<cmtv::HostPool> pool;
  cmtv::PipeConfig pc{32768, 1u << 20, 3, true};
  unsigned threads = 4;
  size_t keyset_cap = 0;
  std::vector<std::pair<std::string, cmtv_keyset*>> keysets;
  std::vector<cmtv_keyset*> evicted;
  std::vector<size_t> live;
  size_t n_devs = 1;
  std::vector<std::vector<FakeSlot>> slots;  // [dev][slot]
  long fail_dev = -1;                        // bulk_wait on this device fails once
  // bulk_wait on this device finds it retired by another call meanwhile (out
  // of live, failed) and fails, once (the pipeline must run on)
  long ext_retire_dev = -1;
  std::vector<bool> failed;
  bool noverify = false;
  uint64_t phase_ns[cmtv::kPhCount] = {};
  cmtv::PipeWorkspace* ws = nullptr;                     // pipebench: every verdict valid, nothing decoded
  uint64_t signatures = 0, invalid = 0, chunks = 0, retired = 0, keyed_chunks = 0;
  std::map<std::string, uint8_t> memo;       // (mode, pk, sig, msg) -> verdict
  std::mutex memo_mu;
  std::map<uintptr_t, size_t> pinned;        // cmtv_alloc_pinned blocks
  uint64_t direct_chunks = 0;
  bool keyset_fail = false;  // registration fails (the pipeline packs direct chunks after all)
  std::atomic<uint64_t> latency_calls{0};
  const uint8_t* guess_pk = nullptr;  // keyset_guess_locked (evicted sets stay allocated until close)
  size_t guess_n = 0;
  const cmtv_keyset* guess_ks = nullptr;
  uint64_t spec_calls = 0, spec_ok = 0;  // speculative launches, and those whose checks held
  uint32_t spec_min = 2048;               // CMTV_SPEC_MIN / CMTV_SPEC at fake_open
  uint64_t masked_chunks = 0;
};

namespace {

struct VecOut {
  std::vector<uint8_t>& v;
  void put(uint32_t pos, uint8_t b) { v[pos] = b; }
  void copy(uint32_t pos, const uint8_t* s, uint32_t len) { std::memcpy(&v[pos], s, len); }
};

uint8_t verify_memo(cmtv_ctx* ctx, uint32_t mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                    size_t mlen) {
  std::string k(1, (char)mode);
  k.append(reinterpret_cast<const char*>(pk), 32);
  k.append(reinterpret_cast<const char*>(sig), 64);
  k.append(reinterpret_cast<const char*>(msg), mlen);
  {
    std::lock_guard<std::mutex> g(ctx->memo_mu);
    auto it = ctx->memo.find(k);
    if (it != ctx->memo.end()) return it->second;
  }
  const uint8_t v = (uint8_t)(oracle_verify_one(pk, msg, mlen, sig, (int)mode) != 0);
  std::lock_guard<std::mutex> g(ctx->memo_mu);
  ctx->memo.emplace(std::move(k), v);
  return v;
}

// verdicts of a templated batch laid out as the device reads it
int device_verify(cmtv_ctx* ctx, size_t n, const uint8_t* keys, bool keyed, const cmtv_keyset* ks, const uint8_t* sig,
                  const uint32_t* off, const cmtv::SbTemplate* tmpls, size_t n_tmpls, const uint8_t* blob,
                  const uint32_t* tidx, const uint8_t* flag, const int64_t* sec, const int32_t* nanos, uint32_t mode,
                  uint8_t* valid) {
  std::vector<uint8_t> msg;
  for (size_t i = 0; i < n; i++) {
    const uint32_t ti = tidx ? tidx[i] : 0u;  // null: one template
    if (ti >= n_tmpls) return CMTV_EINVAL;
    const cmtv::SbTemplate& t = tmpls[ti];
    const uint32_t len = cmtv::sb_msg_len(t, flag[i] != 0, sec[i], nanos[i]);
    if (off[i + 1] - off[i] != len) {
      std::fprintf(stderr, "fake device: message %zu length %u, offsets say %u\n", i, len, off[i + 1] - off[i]);
      return CMTV_EINVAL;
    }
    msg.assign(len, 0);
    VecOut out{msg};
    if (cmtv::sb_write(out, t, blob, flag[i] != 0, sec[i], nanos[i]) != len) return CMTV_EINVAL;
    const uint8_t* pk;
    if (keyed) {
      uint32_t ki = (uint32_t)i;  // null key indices: signature i is by key i
      if (keys) std::memcpy(&ki, keys + 4 * i, 4);
      if (ki >= ks->n) return CMTV_EINVAL;
      pk = ks->pk.data() + 32 * (size_t)ki;
    } else {
      pk = keys + 32 * i;
    }
    valid[i] = verify_memo(ctx, mode, pk, sig + 64 * i, msg.data(), len);
  }
  return CMTV_OK;
}

}  // namespace

namespace cmtv {

int ctx_lock(cmtv_ctx* ctx, std::unique_lock<std::mutex>& lk) {
  lk = std::unique_lock<std::mutex>(ctx->mu);
  return CMTV_OK;
}
void bulk_relock(cmtv_ctx*, std::unique_lock<std::mutex>& lk) { lk.lock(); }
uint32_t ctx_default_mode(const cmtv_ctx*) { return 0; }
bool cache_enabled(const cmtv_ctx*) { return false; }
uint64_t phase_now(const cmtv_ctx*) {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
void phase_add(cmtv_ctx* ctx, int phase, uint64_t t0) { ctx->phase_ns[phase] += phase_now(ctx) - t0; }
void phase_add_ns(cmtv_ctx* ctx, int phase, uint64_t ns) { ctx->phase_ns[phase] += ns; }
bool keyset_cache_enabled(const cmtv_ctx* ctx) { return ctx->keyset_cap != 0; }
int register_keys_locked(cmtv_ctx*, size_t, const uint8_t*, cmtv_keyset**, uint32_t) { return CMTV_EINVAL; }

int verify_host_locked(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                       const uint32_t* msg_off, uint32_t mode, uint8_t* out_valid, uint64_t* out_bitmap) {
  for (size_t i = 0; i < n; i++) {
    const uint8_t v = verify_memo(ctx, mode, pk + 32 * i, sig + 64 * i, msg + msg_off[i], msg_off[i + 1] - msg_off[i]);
    if (out_valid) out_valid[i] = v;
    if (out_bitmap) {
      if ((i & 63) == 0) out_bitmap[i / 64] = 0;
      out_bitmap[i / 64] |= (uint64_t)v << (i & 63);
    }
  }
  ctx->signatures += n;
  return CMTV_OK;
}

int verify_templated_locked(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint32_t* msg_off,
                            const void* tmpls, size_t n_tmpls, const uint8_t* blob, size_t, const uint32_t* tidx,
                            const uint8_t* commit_flag, const int64_t* sec, const int32_t* nanos, uint32_t mode,
                            uint8_t* out_valid, const cmtv_keyset* ks, const uint32_t* key_idx, uint32_t msg_bound,
                            const std::function<bool()>* between, bool* between_ok) {
  ctx->signatures += n;
  if (between) {  // "after the launch" (the fake verifies below)
    *between_ok = (*between)();
    ctx->spec_calls++;
    ctx->spec_ok += *between_ok ? 1 : 0;
  }
  if (ctx->noverify) {  // host-cost runs (pipebench): nothing of the device's work
    std::memset(out_valid, 1, n);
    return CMTV_OK;
  }
  std::vector<uint32_t> off;
  if (msg_off) {
    off.assign(msg_off, msg_off + n + 1);
  } else {
    // offset-free batch (commit.cpp job_prepare_fast): derive them as the
    // real runtime does, and hold the caller to its bound
    off.resize(n + 1);
    uint64_t o = 0;
    const auto* tp = static_cast<const SbTemplate*>(tmpls);
    for (size_t i = 0; i < n; i++) {
      off[i] = (uint32_t)o;
      const uint32_t len = sb_msg_len(tp[tidx ? tidx[i] : 0], commit_flag[i] != 0, sec[i], nanos[i]);
      if (len > msg_bound) return CMTV_EINVAL;
      o += len;
    }
    off[n] = (uint32_t)o;
  }
  return device_verify(ctx, n, ks ? reinterpret_cast<const uint8_t*>(key_idx) : pk, ks != nullptr, ks, sig, off.data(),
                       static_cast<const SbTemplate*>(tmpls), n_tmpls, blob, tidx, commit_flag, sec, nanos, mode,
                       out_valid);
}

const cmtv_keyset* keyset_guess_locked(const cmtv_ctx* ctx, const uint8_t* pk32, size_t n_keys) {
  return ctx->guess_ks && ctx->guess_pk == pk32 && ctx->guess_n == n_keys ? ctx->guess_ks : nullptr;
}
uint32_t spec_min(const cmtv_ctx* ctx) { return ctx->spec_min; }
bool keyset_holds_locked(const cmtv_keyset* ks, const uint8_t* pk32, size_t n_keys) {
  return ks->n == n_keys && std::memcmp(ks->pk.data(), pk32, 32 * n_keys) == 0;
}

const cmtv_keyset* keyset_for_locked(cmtv_ctx* ctx, const uint8_t* pk32, size_t n_keys) {
  if (!ctx->keyset_cap || !n_keys || ctx->keyset_fail) return nullptr;
  std::string key(reinterpret_cast<const char*>(pk32), 32 * n_keys);
  ctx->guess_pk = pk32;
  ctx->guess_n = n_keys;
  for (auto& e : ctx->keysets)
    if (e.first == key) return ctx->guess_ks = e.second;
  auto* ks = new cmtv_keyset();
  ks->n = n_keys;
  ks->pk.assign(pk32, pk32 + 32 * n_keys);
  if (ctx->keysets.size() >= ctx->keyset_cap) {
    // the real cache frees an evicted set once no call has it pinned
    // (runtime.cpp evict_keyset_locked); the fake keeps every one until close
    ctx->evicted.push_back(ctx->keysets.front().second);
    ctx->keysets.erase(ctx->keysets.begin());
  }
  ctx->keysets.emplace_back(std::move(key), ks);
  return ctx->guess_ks = ks;
}

void keyset_pin_locked(const cmtv_keyset* ks) { const_cast<cmtv_keyset*>(ks)->pins++; }
void keyset_unpin_locked(cmtv_ctx*, const cmtv_keyset* ks) { const_cast<cmtv_keyset*>(ks)->pins--; }

std::mutex& bulk_mutex(cmtv_ctx* ctx) { return ctx->bulk_mu; }
HostPool& host_pool(cmtv_ctx* ctx) {
  if (!ctx->pool) ctx->pool.reset(new HostPool(ctx->threads));
  return *ctx->pool;
}
PipeConfig pipe_config(const cmtv_ctx* ctx) {
  PipeConfig pc = ctx->pc;
  pc.chunk_masked = std::max<size_t>(64, pc.chunk * 31 / 32);
  return pc;
}
// latency calls mark the context; the pipeline's chunks after one are masked
// (a flag the fake only counts)
void note_latency(cmtv_ctx* ctx) { ctx->latency_calls++; }
bool call_trace_on(const cmtv_ctx*) { return false; }
uint64_t call_trace_now() { return 0; }
void call_trace_begin_locked(cmtv_ctx*) {}
void call_trace_record_locked(cmtv_ctx*, uint64_t, uint64_t) {}
bool latency_recent(const cmtv_ctx* ctx) { return ctx->latency_calls.load() > 0; }
BulkBusy::BulkBusy(cmtv_ctx* c) : ctx(c) {}
BulkBusy::~BulkBusy() {}
// no streams to swap on the fake devices
LatencyStreams::LatencyStreams(cmtv_ctx* c) : ctx(c) {}
LatencyStreams::~LatencyStreams() {}
int stage_sigs_early_locked(cmtv_ctx*, const uint8_t*, size_t, const uint8_t*) { return CMTV_OK; }
void clear_early_locked(cmtv_ctx*) {}
void live_devices_locked(cmtv_ctx* ctx, std::vector<size_t>& out) { out = ctx->live; }

int bulk_stage(cmtv_ctx* ctx, size_t dev, int slot, const BulkLayout& L, uint8_t** host) {
  FakeSlot& S = ctx->slots[dev][slot];
  if (S.pending) {
    std::fprintf(stderr, "fake: staging of dev %zu slot %d reused while its chunk is in flight\n", dev, slot);
    return CMTV_EHIP;
  }
  // fresh garbage every time: stale bytes from an earlier chunk must not
  // mask a field the host forgot to write (pipebench: grown only, as pinned
  // staging is)
  if (ctx->noverify) {
    if (S.h_in.size() < L.in_bytes) S.h_in.resize(L.in_bytes);
  } else {
    S.h_in.assign(L.in_bytes, 0xA5);
  }
  *host = S.h_in.data();
  return CMTV_OK;
}

// the fake does the whole chunk in bulk_submit_locked
int bulk_prepare(cmtv_ctx*, size_t, int, const BulkLayout&, const cmtv_keyset*) { return CMTV_OK; }
int bulk_submit_locked(cmtv_ctx* ctx, size_t dev, int slot, const BulkLayout& L, const cmtv_keyset* ks,
                       uint32_t mode) {
  FakeSlot& S = ctx->slots[dev][slot];
  if (ctx->failed[dev]) return CMTV_EHIP;  // retired by another call meanwhile
  if (L.in_bytes > S.h_in.size()) return CMTV_EINVAL;
  if (L.direct) {  // the spans must lie in the caller's pinned blocks
    for (int k = 0; k < L.n_spans; k++) {
      const uintptr_t a = reinterpret_cast<uintptr_t>(L.spans[k].host);
      auto it = ctx->pinned.upper_bound(a);
      if (it == ctx->pinned.begin() || a + L.spans[k].bytes > std::prev(it)->first + std::prev(it)->second) {
        std::fprintf(stderr, "fake: span %d outside the pinned blocks\n", k);
        return CMTV_EINVAL;
      }
    }
  }
  S.L = L;
  S.ks = ks;
  if (L.masked) ctx->masked_chunks++;
  S.mode = mode;
  S.pending = true;
  ctx->chunks++;
  ctx->signatures += L.m;
  if (ks) ctx->keyed_chunks++;
  return CMTV_OK;
}

// A direct chunk, as the device sees it (runtime.cpp bulk_submit_locked,
// signbytes.hip k_bulk_gather / k_bulk_bases / k_bulk_rebase): the spans of
// the caller's pinned memory copied to o_arena, then the per-signature layout
// built from the descriptors -- into the slot's buffer, grown to dev_bytes,
// so the packed-chunk reader below checks it the same way.
int bulk_gather(FakeSlot& S) {
  const BulkLayout& L = S.L;
  if (!S.ks || !L.keyed) {
    std::fprintf(stderr, "fake: a direct chunk without registered keys\n");
    return CMTV_EINVAL;
  }
  S.h_in.resize(L.dev_bytes, 0xA5);
  uint8_t* h = S.h_in.data();
  uint8_t* arena = h + L.o_arena;
  for (int k = 0; k < L.n_spans; k++) {
    const BulkSpan& sp = L.spans[k];
    if (sp.dev_off + sp.bytes > L.arena_bytes || (sp.dev_off & 255) != (reinterpret_cast<uintptr_t>(sp.host) & 255)) {
      std::fprintf(stderr, "fake: span %d out of the arena or misaligned\n", k);
      return CMTV_EINVAL;
    }
    std::memcpy(arena + sp.dev_off, sp.host, sp.bytes);
  }
  const auto* desc = reinterpret_cast<const BulkDesc*>(h + L.o_desc);
  const auto* tmpls = reinterpret_cast<const SbTemplate*>(h + L.o_tmpl);
  auto* kidx = reinterpret_cast<uint32_t*>(h + L.o_key);
  auto* off = reinterpret_cast<uint32_t*>(h + L.o_off);
  auto* tidx = reinterpret_cast<uint32_t*>(h + L.o_tidx);
  auto* sec = reinterpret_cast<int64_t*>(h + L.o_sec);
  auto* nanos = reinterpret_cast<int32_t*>(h + L.o_nanos);
  uint64_t o = 0, covered = 0, tmpl_at = 0;
  for (size_t c = 0; c < L.n_tmpls; c++) {
    const BulkDesc& D = desc[c];
    if (!D.m) continue;
    // the templates tile the blob (the plan's lengths are the pack's)
    const SbTemplate& T = tmpls[c];
    if (T.pre_commit_off != tmpl_at || T.pre_nil_off != T.pre_commit_off + T.pre_commit_len ||
        T.post_off != T.pre_nil_off + T.pre_nil_len) {
      std::fprintf(stderr, "fake: template %zu not where the plan put it\n", c);
      return CMTV_EINVAL;
    }
    tmpl_at = T.post_off + T.post_len;
    // the kernel's aligned loads, and every signature once, in order
    if ((D.sig & 7) || (D.sec & 7) || (D.nanos & 3) || D.sp != covered || D.sp + D.m > L.m ||
        D.sig + 64ull * D.m > L.arena_bytes || D.sec + 8ull * D.m > L.arena_bytes ||
        D.nanos + 4ull * D.m > L.arena_bytes || D.flags + D.m > L.arena_bytes) {
      std::fprintf(stderr, "fake: bad descriptor %zu\n", c);
      return CMTV_EINVAL;
    }
    covered += D.m;
    for (uint32_t k = 0; k < D.m; k++) {
      const size_t i = D.sp + k;
      const bool fb = arena[D.flags + k] == 2;
      std::memcpy(h + L.o_sig + 64 * i, arena + D.sig + 64ull * k, 64);
      std::memcpy(&sec[i], arena + D.sec + 8ull * k, 8);
      std::memcpy(&nanos[i], arena + D.nanos + 4ull * k, 4);
      h[L.o_flag + i] = fb ? 1 : 0;
      tidx[i] = (uint32_t)c;
      kidx[i] = k;
      off[i] = (uint32_t)o;
      o += sb_msg_len(tmpls[c], fb, sec[i], nanos[i]);
    }
  }
  if (covered != L.m || o > L.msg_bytes) {
    std::fprintf(stderr, "fake: direct chunk covers %llu of %zu signatures, %llu message bytes (bound %llu)\n",
                 (unsigned long long)covered, L.m, (unsigned long long)o, (unsigned long long)L.msg_bytes);
    return CMTV_EINVAL;
  }
  off[L.m] = (uint32_t)o;
  S.gathered_bytes = o;
  return CMTV_OK;
}

int bulk_wait(cmtv_ctx* ctx, size_t dev, int slot, const uint64_t** bitmap) {
  FakeSlot& S = ctx->slots[dev][slot];
  if (!S.pending) return CMTV_EINVAL;
  S.pending = false;
  if ((long)dev == ctx->fail_dev) {
    ctx->fail_dev = -1;
    return CMTV_EHIP;
  }
  if ((long)dev == ctx->ext_retire_dev) {
    std::lock_guard<std::mutex> g(ctx->mu);  // as the other call would
    ctx->ext_retire_dev = -1;
    ctx->failed[dev] = true;
    for (size_t i = 0; i < ctx->live.size(); i++)
      if (ctx->live[i] == dev) ctx->live.erase(ctx->live.begin() + (long)i);
    ctx->retired++;
    return CMTV_EHIP;
  }
  const BulkLayout& L = S.L;
  if (ctx->noverify) {
    S.bm.assign((L.m + 63) / 64 + 1, ~0ull);
    *bitmap = S.bm.data();
    return CMTV_OK;
  }
  if (L.direct && bulk_gather(S) != CMTV_OK) return CMTV_EINVAL;
  const uint8_t* h = S.h_in.data();
  std::vector<uint8_t> v(L.m);
  const int rc = device_verify(ctx, L.m, h + L.o_key, L.keyed, S.ks, h + L.o_sig,
                               reinterpret_cast<const uint32_t*>(h + L.o_off),
                               reinterpret_cast<const SbTemplate*>(h + L.o_tmpl), L.n_tmpls, h + L.o_blob,
                               reinterpret_cast<const uint32_t*>(h + L.o_tidx), h + L.o_flag,
                               reinterpret_cast<const int64_t*>(h + L.o_sec),
                               reinterpret_cast<const int32_t*>(h + L.o_nanos), S.mode, v.data());
  if (rc != CMTV_OK) return rc;
  const uint32_t* off = reinterpret_cast<const uint32_t*>(h + L.o_off);
  if (off[0] != 0 || off[L.m] != (L.direct ? S.gathered_bytes : L.msg_bytes)) {
    std::fprintf(stderr, "fake: offsets [%u, %u] vs %llu message bytes\n", off[0], off[L.m],
                 (unsigned long long)L.msg_bytes);
    return CMTV_EINVAL;
  }
  // garbage above bit m, as the kernels leave it
  S.bm.assign((L.m + 63) / 64 + 1, 0xDEADBEEFCAFEF00Dull);
  for (size_t i = 0; i < L.m; i++) {
    const uint64_t bit = 1ull << (i & 63);
    S.bm[i / 64] = v[i] ? (S.bm[i / 64] | bit) : (S.bm[i / 64] & ~bit);
  }
  *bitmap = S.bm.data();
  return CMTV_OK;
}

void bulk_drain(cmtv_ctx* ctx) {
  for (auto& d : ctx->slots)
    for (auto& s : d) s.pending = false;
}

bool retire_device_locked(cmtv_ctx* ctx, size_t dev) {
  if (ctx->failed[dev]) return !ctx->live.empty();  // as runtime.cpp
  if (ctx->live.size() < 2) return false;
  ctx->failed[dev] = true;
  for (size_t i = 0; i < ctx->live.size(); i++)
    if (ctx->live[i] == dev) {
      ctx->live.erase(ctx->live.begin() + (long)i);
      ctx->retired++;
      return true;
    }
  return false;
}

void count_invalid_locked(cmtv_ctx* ctx, uint64_t n) { ctx->invalid += n; }
void count_direct_locked(cmtv_ctx* ctx) { ctx->direct_chunks++; }
void pinned_ranges_locked(cmtv_ctx* ctx, std::vector<PinnedRange>& out) {
  out.clear();
  for (auto& b : ctx->pinned) out.push_back(PinnedRange{b.first, b.second});
}
PipeWorkspace*& pipe_workspace(cmtv_ctx* ctx) { return ctx->ws; }

}  // namespace cmtv

// ---- the harness's handle on the fake context
extern "C" cmtv_ctx* fake_open(size_t n_devs, unsigned threads, size_t pipe_min, size_t chunk, int slots,
                               bool pipe_on, size_t keyset_cap, long fail_dev) {
  auto* c = new cmtv_ctx();
  c->n_devs = n_devs;
  c->threads = threads;
  c->pc = cmtv::PipeConfig{pipe_min, chunk, slots, pipe_on};
  c->keyset_cap = keyset_cap;
  c->fail_dev = fail_dev;
  for (size_t d = 0; d < n_devs; d++) c->live.push_back(d);
  c->slots.assign(n_devs, std::vector<FakeSlot>(cmtv::kBulkSlotsMax));
  c->failed.assign(n_devs, false);
  if (const char* v = std::getenv("CMTV_SPEC_MIN")) c->spec_min = (uint32_t)std::max(1l, std::strtol(v, nullptr, 10));
  if (const char* v = std::getenv("CMTV_SPEC")) c->spec_min = v[0] == '0' ? 0 : c->spec_min;
  return c;
}

extern "C" void fake_set_ext_retire(cmtv_ctx* c, long dev) { c->ext_retire_dev = dev; }
extern "C" void fake_set_direct(cmtv_ctx* c, bool on) { c->pc.direct = on; }
extern "C" void fake_set_span(cmtv_ctx* c, uint64_t factor, uint64_t slack) {
  c->pc.span_factor = factor;
  c->pc.span_slack = slack;
}
extern "C" void fake_set_keyset_fail(cmtv_ctx* c, bool on) { c->keyset_fail = on; }

// the ABI's pinned blocks (plain page-aligned memory here)
extern "C" int cmtv_alloc_pinned(cmtv_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out || !bytes) return CMTV_EINVAL;
  void* p = std::aligned_alloc(4096, (bytes + 4095) / 4096 * 4096);
  if (!p) return CMTV_ENOMEM;
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->pinned.emplace(reinterpret_cast<uintptr_t>(p), bytes);
  *out = p;
  return CMTV_OK;
}

extern "C" int cmtv_free_pinned(cmtv_ctx* ctx, void* p) {
  if (!ctx) return CMTV_EINVAL;
  if (!p) return CMTV_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  auto it = ctx->pinned.find(reinterpret_cast<uintptr_t>(p));
  if (it == ctx->pinned.end()) return CMTV_EINVAL;
  ctx->pinned.erase(it);
  std::free(p);
  return CMTV_OK;
}

extern "C" void fake_phases(cmtv_ctx* c, uint64_t* out) {
  for (int p = 0; p < cmtv::kPhCount; p++) out[p] = c->phase_ns[p];
}

extern "C" void fake_set_noverify(cmtv_ctx* c, bool on) { c->noverify = on; }

extern "C" void fake_counts(cmtv_ctx* c, uint64_t* out) {
  out[0] = c->signatures;
  out[1] = c->invalid;
  out[2] = c->chunks;
  out[3] = c->retired;
  out[4] = c->keyed_chunks;
  out[5] = c->direct_chunks;
  out[6] = c->spec_calls;
  out[7] = c->spec_ok;
}

extern "C" void fake_close(cmtv_ctx* c) {
  for (auto& b : c->pinned) std::free(reinterpret_cast<void*>(b.first));
  for (auto& e : c->keysets) delete e.second;
  for (auto* k : c->evicted) delete k;
  cmtv::pipe_workspace_free(c->ws);
  delete c;
}
