// runtime.cpp -- libcmtverify host runtime: contexts over one or more
// devices, streams, pinned staging, sharded kernel launches, the RCCL bitmap
// all-gather and the C ABI of include/cmtverify.h.
//
// A context = one or more devices, each with its own HIP stream, fixed-base
// tables, growable device / pinned buffers and lane-kernel scratch. Calls on a
// context are serialised by its mutex and set the device they touch (cgo
// callers migrate threads). Host-buffer batches are split into contiguous
// 64-aligned shards, one per device, and the shards' verdict bitmaps are
// all-gathered over RCCL (xGMI) when the context has several devices
// (SURVEY.md 8e). There is no CPU verification path: if a device is unusable
// every call fails with a negative code and the caller decides what to do.
#include <dlfcn.h>
#include <sched.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <functional>
#include <memory>
#include <map>
#include <mutex>
#include <new>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/cmtverify.h"
#include "host_pool.h"
#include "kernels.h"
#include "merlin.h"
#include "signbytes.h"
#include "runtime_internal.h"
#include "shard.h"

namespace {

constexpr uint32_t kChunk = 1u << 18;  // signatures per launch (A-table scratch = kChunk * 1280 B)
// registered-key lane launches take up to this many signatures, KB per lane
// (k_verify_keyed_batch, both modes: one field inversion per
// KB signatures; KB = 8 keeps 2,048 waves = two per SIMD); scratch 160 B per
// signature, in the lane kernels' scratch buffer
constexpr uint32_t kKeyedBatchChunk = 1u << 20;
constexpr uint32_t kKeyedBatchMinWaves = 2048;
// The batch-size bands of the verification forms (kernels.h kForm*, picked
// by ed_form / sr_form / keyed_form below), measured on MI355X in round 4 and
// frozen since (no more single-band tuning). CMTV_FORM forces one
// form at every size it can take (tools/*_ab.py use it for A/B runs).
// Ed25519, per call:
//   <= 256     kFormRow4  four waves per signature, one round on 256 CUs
//   <= 1,536   kFormRow   one wave per signature, two workgroups of 3 per CU
//              (profiles/r04_row_max_ab.txt: 1,024 0.215 vs oct2 0.235 ms;
//              2,048: 0.29 vs 0.24 ms)
//   <= 2,048   kFormOct2  eight lanes per signature in two waves
//              (profiles/r04_oct_hs_crossover.txt: 2,048 0.209 vs quad 0.218;
//              3,072 0.272 vs 0.221 ms)
//   <= 49,152  kFormQuad  four rounds of the helper-summed quad kernel
//              (profiles/r04_quad_max_ab.txt: 49,152 0.96 vs lane 1.15 ms;
//              65,536 1.39 vs 1.25 ms)
//   above      kFormLane
// sr25519: the same bands since the round-5 transcript (profiles/
// r05_sr_quad_max_ab.txt: 49,152 0.94 vs lane 1.15 ms; 65,536 1.37 vs 1.25;
// round 4, with the byte-code transcript, crossed at 40,000).
// Registered keys:
//   <= 512     kKeyedRow   (profiles/r04_keyed_row_max_ab.txt: 320-512
//              0.058-0.062 vs quad 0.076 ms; 640-768 lose)
//   <= 36,864  kKeyedQuad  (profiles/r02_keyed_sweep.json: 12,288 per round,
//              0.088/0.164/0.242 ms for 1-3 rounds vs the lane kernel's flat
//              0.28-0.30 ms up to 49k)
//   above      kKeyedLane
constexpr size_t kRow4Max = 256, kRowMax = 1536, kOct2Max = 2048, kQuadMax = 49152, kSrQuadMax = 49152;
constexpr size_t kKeyedRowMax = 512, kKeyedQuadMax = 36864;
constexpr uint32_t kNoForm = 0xFF;
// signatures per device below which a batch is not sharded (env CMTV_SHARD_MIN)
constexpr size_t kShardMinDefault = 8192;
// single-device host batches up to this size return their bitmap through
// mapped host memory (no D2H copy; the writes are a few PCIe transactions),
// and fused commit batches read their staging there (no H2D copy). Measured
// on MI355X (round 4, profiles/r04_zc_max_ab.txt, tools/mid_ab.py, the then knob
// 4,096 vs 16,384): VerifyCommit at 8,192 0.329-0.330 -> 0.320 ms, at 10,000
// 0.349 -> 0.341-0.343 ms; the host API unchanged. 4,096 before.
constexpr size_t kZeroCopyMax = 12288;
// tagged bitmap entries of a polled host batch (CmtvDev::h_tags): a row
// launch's 32-signature words or a keyed quad launch's 16-signature slices
constexpr size_t kTagEntries = std::max<size_t>(cmtv::kRowMaxCap / 32 + 1, 4 * ((kZeroCopyMax + 63) / 64));
constexpr int kMaxDevices = 64;

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    want = want + want / 4;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    want = want + want / 4;
    hipError_t e = hipHostMalloc(&p, want, flags);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Lane-kernel scratch (the generic kernel's A tables, the batched keyed
// kernel's R' and Z products) and the event of its last user: a launch on
// another stream waits for that user (acquire_scratch), growing it first
// waits for it to finish.
struct Scratch {
  DevBuf buf;
  hipEvent_t done = nullptr;
  bool used = false;
};

// SipHash-2-4 (Aumasson & Bernstein), keyed per process: the verdict cache's
// index, so a peer cannot aim many entries at one bucket.
uint64_t rotl(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

struct SipKey {
  uint64_t k0, k1;
  SipKey() {
    std::random_device rd;
    k0 = ((uint64_t)rd() << 32) ^ rd();
    k1 = ((uint64_t)rd() << 32) ^ rd();
  }
};

uint64_t siphash24(const SipKey& key, const uint8_t* p, size_t n) {
  uint64_t v0 = 0x736f6d6570736575ull ^ key.k0, v1 = 0x646f72616e646f6dull ^ key.k1;
  uint64_t v2 = 0x6c7967656e657261ull ^ key.k0, v3 = 0x7465646279746573ull ^ key.k1;
  auto round = [&] {
    v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);
    v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;
    v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;
    v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);
  };
  const size_t full = n & ~(size_t)7;
  for (size_t i = 0; i < full; i += 8) {
    uint64_t m;
    std::memcpy(&m, p + i, 8);
    v3 ^= m;
    round();
    round();
    v0 ^= m;
  }
  uint64_t b = (uint64_t)n << 56;
  for (size_t i = full; i < n; i++) b |= (uint64_t)p[i] << (8 * (i - full));
  v3 ^= b;
  round();
  round();
  v0 ^= b;
  v2 ^= 0xff;
  round();
  round();
  round();
  round();
  return v0 ^ v1 ^ v2 ^ v3;
}

// Verdict cache (cmtv_verdict_cache): a ring of the last `cap` verdicts,
// indexed by a keyed hash of the full key (scheme + mode, pk, sig, msg); a hit
// also compares the key bytes, so it returns exactly the device verdict.
struct VerdictCache {
  struct Entry {
    std::string key;
    uint64_t h = 0;
    uint8_t verdict = 0;
    bool used = false;
  };
  SipKey sk;
  size_t cap = 0;
  size_t next = 0;
  std::vector<Entry> ring;
  std::unordered_multimap<uint64_t, size_t> index;

  uint64_t hash(const std::string& k) const {
    return siphash24(sk, reinterpret_cast<const uint8_t*>(k.data()), k.size());
  }
  static void make_key(std::string& k, uint32_t mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                       size_t mlen) {
    k.resize(1 + 32 + 64 + mlen);
    k[0] = (char)(mode == cmtv::kModeSr25519 ? 0x80 : mode);  // scheme + verdict mode
    std::memcpy(&k[1], pk, 32);
    std::memcpy(&k[33], sig, 64);
    if (mlen) std::memcpy(&k[97], msg, mlen);
  }
  void reset(size_t c) {
    cap = c;
    next = 0;
    ring.clear();
    ring.resize(c);
    index.clear();
  }
  // verdict or -1
  int find(uint64_t h, const std::string& k) const {
    auto r = index.equal_range(h);
    for (auto it = r.first; it != r.second; ++it)
      if (ring[it->second].key == k) return ring[it->second].verdict;
    return -1;
  }
  void insert(uint64_t h, std::string&& k, uint8_t v) {
    if (!cap) return;
    Entry& e = ring[next];
    if (e.used) {
      auto r = index.equal_range(e.h);
      for (auto it = r.first; it != r.second; ++it)
        if (it->second == next) {
          index.erase(it);
          break;
        }
    }
    e.key = std::move(k);
    e.h = h;
    e.verdict = v;
    e.used = true;
    index.emplace(h, next);
    next = (next + 1) % cap;
  }
  size_t size() const { return index.size(); }
};

// ---------------------------------------------------------------- RCCL (dlopen)
// Resolved at run time with RTLD_LOCAL so the library loads (and a context
// falls back to peer copies) where librccl is absent, and so RCCL's symbols
// never interpose on a host process that carries its own copy.
typedef void* ncclComm_t;
typedef int ncclResult_t;
constexpr int kNcclUint64 = 5;  // ncclDataType_t ncclUint64 (rccl.h)

struct Rccl {
  bool ok = false;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;  // optional (a failed group's stuck ranks)
};

Rccl load_rccl(const char* path) {
  Rccl x;
  void* h = nullptr;
  if (path) {
    h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  } else {
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
  }
  if (!h) return x;
  x.CommInitAll = reinterpret_cast<decltype(x.CommInitAll)>(dlsym(h, "ncclCommInitAll"));
  x.CommDestroy = reinterpret_cast<decltype(x.CommDestroy)>(dlsym(h, "ncclCommDestroy"));
  x.AllGather = reinterpret_cast<decltype(x.AllGather)>(dlsym(h, "ncclAllGather"));
  x.GroupStart = reinterpret_cast<decltype(x.GroupStart)>(dlsym(h, "ncclGroupStart"));
  x.GroupEnd = reinterpret_cast<decltype(x.GroupEnd)>(dlsym(h, "ncclGroupEnd"));
  x.CommAbort = reinterpret_cast<decltype(x.CommAbort)>(dlsym(h, "ncclCommAbort"));
  x.ok = x.CommInitAll && x.CommDestroy && x.AllGather && x.GroupStart && x.GroupEnd;
  return x;
}

// The RCCL entry points for a context: the system librccl, or the library
// CMTV_RCCL_LIB names (read at open; tests/host/rccl_stub.cpp rehearses the
// multi-rank code on one GPU). Each library is resolved once per process.
const Rccl& rccl(const std::string& path = std::string()) {
  static std::mutex mu;
  static std::unordered_map<std::string, Rccl> libs;
  std::lock_guard<std::mutex> g(mu);
  auto it = libs.find(path);
  if (it == libs.end()) it = libs.emplace(path, load_rccl(path.empty() ? nullptr : path.c_str())).first;
  return it->second;
}

// Kernel timing: HIP event pairs recorded around each verification on its
// stream, harvested without blocking once complete (so device-resident calls
// stay asynchronous).
struct Timing {
  struct Pair {
    hipEvent_t a = nullptr, b = nullptr;
  };
  std::vector<Pair> free_;
  std::deque<Pair> pending;
  // pairs in flight beyond this are not timed (begin hands out a null pair)
  static constexpr size_t kMaxPending = 1u << 16;
  hipError_t begin(Pair& p, hipStream_t s) {
    if (pending.size() >= kMaxPending) {
      p = Pair();
      return hipSuccess;
    }
    if (free_.empty()) {
      Pair q;
      hipError_t e = hipEventCreate(&q.a);
      if (e == hipSuccess) e = hipEventCreate(&q.b);
      if (e != hipSuccess) return e;
      free_.push_back(q);
    }
    p = free_.back();
    free_.pop_back();
    hipError_t e = hipEventRecord(p.a, s);
    if (e != hipSuccess) free_.push_back(p);
    return e;
  }
  hipError_t end(const Pair& p, hipStream_t s) {
    if (!p.a) return hipSuccess;  // untimed (kMaxPending)
    hipError_t e = hipEventRecord(p.b, s);
    if (e != hipSuccess) {
      free_.push_back(p);
      return e;
    }
    pending.push_back(p);
    return hipSuccess;
  }
  void abandon(const Pair& p) {
    if (p.a) free_.push_back(p);
  }
  // completed pairs -> stats (context-wide and this device's); blocking
  // waits for all of them
  void harvest(cmtv_stats& st, double& dev_ms, uint64_t& dev_timed, bool blocking) {
    while (!pending.empty()) {
      Pair p = pending.front();
      // never blocks unless asked (cmtv_stats_get): a device-resident call
      // must not wait for launches parked on other streams
      if (blocking) {
        if (hipEventSynchronize(p.b) != hipSuccess) break;
      } else if (hipEventQuery(p.b) != hipSuccess) {
        break;
      }
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
        st.last_kernel_ms = ms;
        st.device_ms += ms;
        st.timed_calls++;
        dev_ms += ms;
        dev_timed++;
      }
      pending.pop_front();
      free_.push_back(p);
    }
  }
  void release() {
    for (auto& p : pending) free_.push_back(p);
    pending.clear();
    for (auto& p : free_) {
      if (p.a) (void)hipEventDestroy(p.a);
      if (p.b) (void)hipEventDestroy(p.b);
    }
    free_.clear();
  }
};

}  // namespace

// A device's bulk lane (runtime_internal.h): staging slots and streams of
// the cross-height pipeline.
struct BulkSlot {
  HostBuf h_in;   // pinned staging, packed by the host workers
  // verdict bitmap: D2H'd into it, or (registered-key chunks) written there
  // by the kernel itself (coherent, mapped)
  HostBuf h_bm{nullptr, 0, hipHostMallocCoherent | hipHostMallocMapped};
  DevBuf d_in;    // the staging on the device, then the sign-bytes
  DevBuf d_bm;    // verdict bitmap
  hipEvent_t h2d = nullptr, done = nullptr;
  hipEvent_t prep = nullptr;  // the chunk's gather + sign-bytes done (BulkLane::prep)
  bool pending = false;  // submitted, not yet waited for
};
struct BulkLane {
  hipStream_t copy = nullptr, exec = nullptr;
  // the exec stream of chunks submitted near a latency call: every CU but
  // the reserved ones (its own hardware queue, cu_mask), and the waves one
  // round of it holds at two per SIMD (the keyed batch kernel's occupancy)
  hipStream_t exec_masked = nullptr;
  // (unused: a fifth hardware queue per lane cost the latency calls beside a
  // pipeline ~70 us of p99 -- round 6, profiles/r06_prep_queue_ab.txt; an
  // unmasked chunk's prep runs on exec_masked instead, bulk_prep_stream)
  hipStream_t prep = nullptr;
  // ... and the device's latency stream while a pipeline call is in flight
  // (LatencyStreams): the reserved CUs only, so a 150-validator commit's
  // workgroups never share a CU -- its SIMDs, its instruction cache (one per
  // CU pair) -- with the bulk launch's waves; lat_in / lat_out order it
  // after / before the device's normal stream
  hipStream_t lat = nullptr;
  hipEvent_t lat_in = nullptr, lat_out = nullptr;
  uint32_t cus = 0, masked_waves = 0;
  BulkSlot slot[cmtv::kBulkSlotsMax];
  Scratch scratch;
};

// Per-device state of a context.
struct CmtvDev {
  int ordinal = 0;
  hipStream_t stream = nullptr;
  uint32_t* d_btab = nullptr;
  uint32_t* d_srprog = nullptr;  // sr25519 transcript: the sponge after the constant prefix (merlin.h)
  DevBuf d_in, d_out, d_all;
  HostBuf h_in, h_out;
  // small single-device host batches: the kernel writes the verdict bitmap
  // straight into this coherent, device-mapped host buffer (no D2H copy)
  HostBuf h_zc{nullptr, 0, hipHostMallocCoherent | hipHostMallocMapped};
  // ... and, with fused sign-bytes, reads its inputs straight from this one
  // (no H2D copy, no copy-engine -> compute dependency before the kernel)
  HostBuf h_zin{nullptr, 0, hipHostMallocCoherent | hipHostMallocMapped};
  // The lane kernels' A-table scratch is shared by every launch on this
  // device, whatever stream it is enqueued on: each lane launch waits for the
  // previous one (Scratch::done) so calls on different streams cannot
  // overwrite each other's tables. (The bulk lane has its own.)
  Scratch scratch;
  hipEvent_t done = nullptr;  // cross-device ordering for peer-copy gathers
  Timing timing;
  ncclComm_t comm = nullptr;
  // kernel diagnostic counters (kernels.h kDiagWords, vector atomics)
  uint32_t* d_diag = nullptr;
  // the row kernel's bitmap ring (kernels.h kRowSlots x kRowSlotWords)
  uint32_t* d_rowslots = nullptr;
  uint32_t row_seq = 0;
  // per ring slot: an event recorded after the device-resident launch that
  // last took it (row_pending), waited on before the slot is handed out again
  // (row_slot_acquire), so a slot is never shared by two launches in flight
  hipEvent_t row_ev[cmtv::kRowSlots] = {};
  bool row_pending[cmtv::kRowSlots] = {};
  // the row kernels' tagged bitmap (kernels.h RowSlot) for small host
  // batches: run_host_batch_ arms tag_arm (h_tags' device pointer) and a fresh
  // tag_seq around its launch; a row launch that takes them sets tag_used, and
  // the call polls the entries (wait_row_tags) instead of synchronising the
  // stream
  HostBuf h_tags{nullptr, 0, hipHostMallocCoherent | hipHostMallocMapped};
  uint64_t* d_tags = nullptr;
  uint64_t* tag_arm = nullptr;
  uint32_t tag_seq = 0;
  bool tag_used = false;
  // signatures per tagged entry of the launch that took the tags: 32 (row
  // kernels' words) or 16 (the keyed quad kernel's per-wave slices)
  uint32_t tag_width = 32;
  // A polled host call returns once its tags are in, while the row launch
  // may still be retiring (its last waves zero their ring words). poll_ev is
  // recorded after that launch; the next host call on the device -- before it
  // writes the mapped staging (h_zin) the launch read -- and the next row-slot
  // acquisition wait for it (settle_polled), so neither the staging nor a ring
  // slot is ever shared with a launch still in flight.
  hipEvent_t poll_ev = nullptr;
  bool poll_pending = false;
  // signatures a single-commit call copied to h_in / d_in (offset 0) before
  // planning (stage_sigs_early_locked): the source and count, and the keys
  // copied after them (generic kernels; null when none); the next staging of
  // those bytes skips them
  const uint8_t* early_src = nullptr;
  const uint8_t* early_pk = nullptr;
  size_t early_n = 0;
  // a device that returned a HIP error is taken out of the context's
  // rotation: host batches are re-planned over the others (runtime.cpp
  // run_host_batch); CMTV_FAULT_DEV=g makes device g's first launch fail
  bool failed = false;
  bool inject_fault = false;
  // this device's share of cmtv_stats (cmtv_device_stats_get)
  uint64_t calls = 0, signatures = 0, launches = 0, timed_calls = 0;
  double device_ms = 0;
  // verification calls on this device (CMTV_TIMING samples one in timing_every)
  uint64_t timing_seq = 0;
  BulkLane bulk;  // the pipeline's lane on this device (created on first use)
};

struct cmtv_ctx {
  std::vector<CmtvDev> devs;  // devs[0]: single-device and device-resident calls
  bool rccl = false;          // gathers over an RCCL communicator
  uint32_t default_mode = CMTV_MODE_GO_STDLIB;
  std::mutex mu;
  cmtv_stats stats{};
  // CMTV_FORM: a form forced at every size it can take (kNoForm: the bands)
  uint32_t force_form = kNoForm, force_keyed = kNoForm;
  uint32_t hs_tune = 0;  // CMTV_HS_PRE + 1 (bits 0..7); 0: the kernel's default
  size_t lane_chunk = kChunk;         // signatures per lane-kernel launch (env CMTV_LANE_CHUNK)
  size_t shard_min = kShardMinDefault;
  int sr_nops = 0;
  VerdictCache cache;                 // cmtv_verdict_cache (off by default)
  // cmtv_keyset_cache: validator sets (their concatenated keys) -> registered
  // key sets, used by cmtv_verify_commit(s); FIFO of at most keyset_cap
  size_t keyset_cap = 0;
  std::vector<std::pair<std::string, cmtv_keyset*>> keysets;
  // CMTV_FAULT_AT: 1-based index of the verification launch that fails
  uint64_t fault_at = 0, launch_seq = 0;
  bool fault_pending = false;  // the last failure was CMTV_FAULT_AT's
  // RCCL options read at open (CMTV_FORCE_RCCL, CMTV_NO_RCCL) and the
  // library to load (CMTV_RCCL_LIB; empty: the system librccl)
  bool force_rccl = false, no_rccl = false, no_rccl_fallback = false;
  std::string rccl_lib;
  // a gather failed inside RCCL: the context never builds a communicator
  // again (rebuild_comm after a device retirement included); gathers use
  // peer copies. rccl_drain_ms bounds the wait for the failed group's
  // streams (CMTV_RCCL_DRAIN_MS): a rank whose collective was enqueued before
  // the group failed never completes without its peers.
  bool rccl_broken = false;
  uint32_t rccl_drain_ms = 2000;
  // CMTV_FORCE_WIDE: quad kernels take the 64-window half-scalar fallback
  bool force_wide = false;
  // templated sign-bytes in the split kernels' helper waves (CMTV_NO_SB_FUSE=1: off)
  bool sb_fuse = true;
  // polls of the keyed split kernel's quads for the hash helper's k before
  // they hash themselves (CMTV_FORCE_K_LATE=1: 0, every quad wave hashes)
  uint32_t keyed_wait = cmtv::kKeyedWaitDefault;
  // waves a batched launch must keep (CMTV_KEYED_BATCH_MIN_WAVES; 1 batches
  // any size, the test knob that puts the corpus through the batched kernels)
  uint32_t keyed_batch_min_waves = kKeyedBatchMinWaves;
  // devices (indices into devs) that take host batches, in shard order; the
  // RCCL communicator (when rccl) spans exactly these, rank = position
  std::vector<size_t> live;
  // fused small host batches read their inputs from mapped host memory (CMTV_NO_ZC_IN=1: off)
  bool zc_in = true;
  bool zc_host_in = true;  // CMTV_ZC_HOST_IN=0: host-API batches copy their staging to HBM
  bool early_sigs = true;  // CMTV_EARLY_SIGS=0: a commit's signatures are staged after its plan
  // single-device host batches up to this size take the mapped-memory path
  size_t zc_max = kZeroCopyMax;
  // small host batches on a row kernel poll its tagged bitmap words
  // (run_host_batch_); CMTV_HOST_POLL=0 synchronises the stream
  bool host_poll = true;
  // set while a host-buffer call runs (run_host_batch): its launches finish
  // before the call returns, so their row-ring slots need no fence event
  bool host_sync = false;
  // CMTV_ROW_FENCE=0: no row-ring fence (only for the test that shows the race)
  bool row_fence = true;
  // kernel timing by HIP event pairs on one call in timing_every per device
  // (cmtv_stats device_ms / timed_calls; CMTV_TIMING=N, 0: off). The pair's
  // marker packets cost ~4 us of a 150-validator call and ~8 us between
  // back-to-back 10k launches (tools/step_gap.py), so not every call pays.
  uint32_t timing_every = 16;
  // CMTV_HOST_PHASES=1: host phase clock (runtime_internal.h HostPhase)
  bool phases_on = false;
  uint64_t phase_ns[cmtv::kPhCount] = {};
  uint64_t phase_calls = 0;
  // CMTV_FAULT_SYNC_DEV=g: device g's stream synchronisation in a host batch
  // reports a HIP error (a fault found after the launch; re-shard test knob)
  long fault_sync_dev = -1;
  // the cross-height pipeline (pipeline.cpp): its bulk lanes and worker pool
  // belong to the holder of bulk_mu; cmtv_verify_commits calls of at least
  // pipe_min signatures take it (CMTV_PIPE_MIN; CMTV_PIPELINE=0: never),
  // in chunks of about pipe_chunk signatures (CMTV_PIPE_CHUNK) over
  // pipe_slots staging slots per device (CMTV_PIPE_SLOTS), on host_threads
  // threads (CMTV_HOST_THREADS; default: the CPUs this process may use, less
  // 3 when more than 8, at most 16: host_pool)
  std::mutex bulk_mu;
  std::unique_ptr<cmtv::HostPool> pool;
  unsigned host_threads = 0;
  size_t pipe_min = 32768, pipe_chunk = 1u << 20;
  int pipe_slots = 3;
  bool pipe_on = true;
  bool pipe_direct = true;  // CMTV_PIPE_DIRECT=0: pinned arguments are packed too
  // Latency calls beside a pipeline (a 150-validator
  // VerifyCommit from consensus while blocksync replays): a pipeline chunk
  // submitted within lat_window_ns of such a call (cmtv_verify_commit, a
  // small one-batch cmtv_verify_commits or host batch: note_latency) runs on
  // the lane's CU-masked exec stream, which leaves lat_reserve_cus CUs (one
  // per 32) to the device's normal stream, and is cut to what the other CUs
  // hold in one round; while a pipeline call is in flight (bulk_busy) the
  // latency call takes a form that fits those CUs (under_load, snapshotted at
  // each lock hold). CMTV_LAT_WINDOW_MS (default 10,000; 0: never masked),
  // CMTV_LAT_RESERVE_CUS (default 16); CMTV_LOAD_FORM=0 keeps the latency
  // call's idle form under load.
  std::atomic<uint64_t> last_latency_ns{0};
  bool load_form = true;
  // a pipeline call is in flight (snapshotted with under_load): a registered-
  // key latency batch then reads its staging in place (mapped host memory)
  // rather than queue its H2D copy on the copy engines behind the pipeline's
  // chunk DMAs; CMTV_LOAD_ZC=0 copies it as when idle
  bool bulk_now = false, load_zc = true;
  // ... and waits for its stream rather than polling its kernel's tagged
  // bitmap (run_host_batch_; CMTV_LOAD_POLL=1 polls as when idle)
  bool load_nopoll = true;
  // the quad kernels' tagged slices (CMTV_QUAD_POLL=1): polling a 10k commit
  // was slower than waiting for its stream on MI355X (round 6,
  // tools/gpu_r6p.sh, three alternating rounds: keyset pinned p50 0.112-0.119
  // polled vs 0.108-0.110 ms, generic 0.269-0.279 vs 0.267 ms), so off
  bool quad_poll = false;
  // registered-key small batches read their staging in place -- signatures in
  // the caller's cmtv_alloc_pinned memory straight from there -- instead of
  // an early signature DMA + the split staging (CMTV_KEYED_ZC=0). Measured
  // on MI355X (round 6, tools/gpu_r6x.sh, three alternating rounds):
  // verify_commit_10k_keyset pinned p50 0.105 / 0.1085 / 0.1051 against
  // 0.1118 / 0.1074 / 0.108 ms, heap 0.114-0.117 against 0.117-0.123 ms
  bool keyed_zc = true;
  bool spin_wait = false;  // CMTV_SPIN_WAIT (wait_stream)
  bool prep_stream = true;  // CMTV_PREP_STREAM (BulkLane::prep)
  bool one_exec = false;    // CMTV_ONE_EXEC (bulk_lane_init)
  // CMTV_BULK_BM_DIRECT=1 (bulk_submit_locked): off -- two alternating rounds
  // (profiles/r06_bm_direct_ab.txt) gave VerifyCommit -0.13 ms but
  // VerifyCommitLight +0.5-0.7 ms per pass
  bool bulk_bm_direct = false;
  bool split_submit = true;  // CMTV_SPLIT_SUBMIT (PipeConfig::split_submit)
  // CMTV_CALL_TRACE=1 (diagnostics): per single-commit call, the time to the
  // context lock, to the launch, to the verdicts and to the return; their
  // percentiles printed on stderr at cmtv_close
  bool call_trace = false, call_trace_loaded_only = false;
  uint64_t trace_launch = 0, trace_wait = 0;  // this hold's marks (lock held)
  uint64_t trace_dev_ns = 0;
  hipEvent_t trace_ev[2] = {nullptr, nullptr};
  std::mutex trace_mu;
  std::vector<std::array<uint64_t, 5>> trace_rows;
  uint64_t lat_window_ns = 10'000'000'000ull;
  uint32_t lat_reserve_cus = 16;
  // latency calls beside a pipeline run on the reserved CUs only
  // (LatencyStreams; CMTV_LAT_ISOLATE=0: on the whole device, beside the
  // bulk waves)
  bool lat_isolate = true;
  std::atomic<int> bulk_busy{0};
  // threads blocked in ctx_lock: a pipeline re-taking the lock for its next
  // chunk lets them in first (bulk_relock)
  std::atomic<int> lock_waiters{0};
  bool under_load = false;
  uint32_t cus = 0;  // CUs per device (the smallest of the context's)
  // the caller's pinned blocks (cmtv_alloc_pinned): base -> bytes; chunks
  // whose arrays lie in one are DMA'd from it (pipeline.cpp direct chunks)
  std::map<uintptr_t, size_t> pinned;
  // the last key set keyset_for_locked returned, by the caller's key array
  // (commit.cpp's speculative VerifyCommit launches with it, and checks the
  // keys' bytes while the kernel runs); cleared when that set is evicted
  uint32_t spec_min = 2048;  // CMTV_SPEC_MIN; CMTV_SPEC=0: 0 (off)
  const uint8_t* guess_pk = nullptr;
  size_t guess_n = 0;
  const cmtv_keyset* guess_ks = nullptr;
  // cached key sets evicted while a pipeline call had them pinned
  std::vector<cmtv_keyset*> zombies;
  cmtv::PipeWorkspace* pipe_ws = nullptr;
};

struct cmtv_keyset {
  struct PerDev {
    uint32_t* d_pk = nullptr;   // n x 8 words, the keys' original bytes
    uint8_t* d_ok = nullptr;    // n decode flags
    uint32_t* d_tab = nullptr;  // n x kCombWords
    uint32_t* d_wide = nullptr; // n x kWideTableWords (CMTV_KEYS_WIDE), else null
  };
  cmtv_ctx* ctx = nullptr;
  size_t n = 0;
  int pins = 0;               // pipeline calls using this cached set
  bool evicted = false;       // left the keyset cache while pinned
  std::vector<PerDev> dev;    // one per device of the context
  std::vector<uint8_t> pk;    // host copy (n x 32)
};

namespace cmtv {

static void evict_keyset_locked(cmtv_ctx* ctx, cmtv_keyset* ks);

static int hip_fail(hipError_t e) {
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return CMTV_ENOMEM;
  return CMTV_EHIP;
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

uint64_t phase_now(const cmtv_ctx* ctx) {
  if (!ctx->phases_on) return 0;
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void phase_add(cmtv_ctx* ctx, int phase, uint64_t t0) {
  if (!ctx->phases_on || !t0) return;
  ctx->phase_ns[phase] += phase_now(ctx) - t0;
  if (phase == kPhPrepare) ctx->phase_calls++;
}

void phase_add_ns(cmtv_ctx* ctx, int phase, uint64_t ns) {
  if (!ctx->phases_on) return;
  ctx->phase_ns[phase] += ns;
  if (phase == kPhPipePlan) ctx->phase_calls++;
}

static void harvest(cmtv_ctx* ctx, bool blocking) {
  for (auto& d : ctx->devs) {
    if (d.failed) continue;
    (void)hipSetDevice(d.ordinal);
    d.timing.harvest(ctx->stats, d.device_ms, d.timed_calls, blocking);
  }
}

// CMTV_FAULT_AT: true when this verification launch is the one to fail
static bool fault_hit(cmtv_ctx* ctx) {
  ctx->launch_seq++;
  if (ctx->fault_at && ctx->launch_seq == ctx->fault_at) {
    ctx->stats.faults_injected++;
    ctx->fault_pending = true;
    return true;
  }
  return false;
}

// A lane launch's scratch (Scratch: a device's, shared by every stream, or
// the bulk lane's): the launch waits for the previous user, growing it first
// waits for that user to finish.
static hipError_t acquire_scratch(Scratch& S, size_t bytes, hipStream_t s) {
  hipError_t e;
  if (bytes > S.buf.cap) {
    // growing frees the old scratch: every earlier user must be done
    if (S.used && (e = hipEventSynchronize(S.done)) != hipSuccess) return e;
    if ((e = S.buf.ensure(bytes)) != hipSuccess) return e;
  }
  if (S.used && (e = hipStreamWaitEvent(s, S.done, 0)) != hipSuccess) return e;
  return hipSuccess;
}

static hipError_t release_scratch(Scratch& S, hipStream_t s) {
  const hipError_t e = hipEventRecord(S.done, s);
  if (e == hipSuccess) S.used = true;
  return e;
}

// Waits for the last polled host launch on D (CmtvDev::poll_ev); it has
// normally retired by then, so this is one event query.
static hipError_t settle_polled(CmtvDev& D) {
  if (!D.poll_pending) return hipSuccess;
  hipError_t e = hipEventQuery(D.poll_ev);
  if (e == hipErrorNotReady) e = hipEventSynchronize(D.poll_ev);
  if (e == hipSuccess) D.poll_pending = false;
  return e;
}

// The row kernels' verdict-byte ring (kernels.h kRowSlots): the next slot for
// a launch on stream s. The kernel's last wave packs the bitmap from the slot
// and resets its counter, so two launches in flight on one slot would count
// each other's waves. A slot whose last user was a device-resident launch
// (enqueued on a caller's stream, not waited for before its call returned) is
// fenced: s waits for that launch's event. Host-buffer calls finish their
// launches before they return (ctx->host_sync) and record nothing.
// With a bitmap, a launch of an armed host batch also takes the tagged bitmap
// (CmtvDev::tag_arm). Each entry is stored after its slot word is zero again,
// so a slot needs no fence against a tagged launch still retiring.
static hipError_t row_slot_acquire(cmtv_ctx* ctx, CmtvDev& D, hipStream_t s, bool bitmap, RowSlot& slot,
                                   uint32_t& k) {
  hipError_t e0 = settle_polled(D);
  if (e0 != hipSuccess) return e0;
  k = D.row_seq++ % kRowSlots;
  slot = RowSlot{};
  slot.words = D.d_rowslots + (size_t)k * kRowSlotWords;
  if (bitmap && D.tag_arm) {
    slot.tagged = D.tag_arm;
    slot.seq = D.tag_seq;
    D.tag_used = true;
    D.tag_width = 32;
  }
  if (!D.row_pending[k] || !ctx->row_fence) return hipSuccess;
  hipError_t e = hipEventQuery(D.row_ev[k]);
  if (e == hipErrorNotReady) e = hipStreamWaitEvent(s, D.row_ev[k], 0);
  if (e != hipSuccess) return e;
  D.row_pending[k] = false;
  return hipSuccess;
}

static hipError_t row_slot_release(cmtv_ctx* ctx, CmtvDev& D, hipStream_t s, uint32_t k) {
  if (ctx->host_sync || !ctx->row_fence) return hipSuccess;
  hipError_t e = hipSuccess;
  if (!D.row_ev[k]) e = hipEventCreateWithFlags(&D.row_ev[k], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventRecord(D.row_ev[k], s);
  if (e == hipSuccess) D.row_pending[k] = true;
  return e;
}

// The form of a batch of n Ed25519 signatures (the bands above, or CMTV_FORM
// where the forced form can take n: a row form at most kRowMaxCap in one launch)
static uint32_t ed_form(const cmtv_ctx* ctx, size_t n) {
  const uint32_t f = ctx->force_form;
  if (f != kNoForm && !((f == kFormRow || f == kFormRow4) && n > kRowMaxCap)) return f;
  // beside a running pipeline only its reserved CUs are free: 48 signatures
  // per workgroup (quad) rather than one (row) or eight (oct)
  if (ctx->under_load && n <= kQuadMax) return kFormQuad;
  return n <= kRow4Max ? kFormRow4 : n <= kRowMax ? kFormRow : n <= kOct2Max ? kFormOct2 : n <= kQuadMax ? kFormQuad
                                                                                                       : kFormLane;
}

// ... of sr25519 signatures (the quad and lane forms)
static uint32_t sr_form(const cmtv_ctx* ctx, size_t n) {
  const uint32_t f = ctx->force_form;
  if (f == kFormQuad || f == kFormLane) return f;
  return n <= kSrQuadMax ? kFormQuad : kFormLane;
}

// ... and of registered-key signatures
static uint32_t keyed_form(const cmtv_ctx* ctx, size_t n) {
  const uint32_t f = ctx->force_keyed;
  if (f != kNoForm && !(f == kKeyedRow && n > kRowMaxCap)) return f;
  if (ctx->under_load && n <= kKeyedQuadMax) return kKeyedQuad;  // as ed_form
  return n <= kKeyedRowMax ? kKeyedRow : n <= kKeyedQuadMax ? kKeyedQuad : kKeyedLane;
}

// The forms whose helper wave can write templated sign-bytes itself
// (kernels.h SbFuse) when they run in one launch (enqueue_verify rejects a
// fused batch of more than kChunk): every form but the lane kernels. The one
// predicate enqueue_shard and the enqueue functions use.
static bool fuse_ok(const cmtv_ctx* ctx, size_t n) { return ed_form(ctx, n) != kFormLane && n <= kChunk; }
static bool keyed_fuse_ok(const cmtv_ctx* ctx, size_t n) { return keyed_form(ctx, n) != kKeyedLane && n <= kChunk; }

// Enqueue verification of n signatures whose inputs are in device memory of
// device D (current on this thread).
static int enqueue_verify(cmtv_ctx* ctx, CmtvDev& D, size_t n, const uint8_t* d_pk, const uint8_t* d_sig,
                          const uint8_t* d_msg, const uint32_t* d_off, uint32_t mode, uint8_t* d_valid,
                          uint64_t* d_bitmap, hipStream_t s, const SbFuse* sb = nullptr, Scratch* scr = nullptr) {
  Scratch& S = scr ? *scr : D.scratch;
  if (n == 0) return CMTV_OK;
  if (fault_hit(ctx) || D.inject_fault) return CMTV_EHIP;
  // fused sign-bytes only where the split kernels run, in one launch
  if (sb && (mode == kModeSr25519 || !fuse_ok(ctx, n))) return CMTV_EINVAL;
  // Small batches cannot fill the chip at one signature per lane: more lanes
  // per signature below the bands' crossovers (quad.h, oct.h, row.h,
  // sr25519_quad.h)
  const bool sr = mode == kModeSr25519;
  const uint32_t form = sr ? sr_form(ctx, n) : ed_form(ctx, n);
  const bool lane = form == kFormLane;
  const bool row = form == kFormRow || form == kFormRow4;
  const uint32_t kflags = form | (form == kFormQuad ? ctx->hs_tune << 16 : 0u) |
                          (ctx->force_wide ? kLaunchForceWide : 0u);
  hipError_t e = hipSuccess;
  if (lane) {
    const size_t lanes = std::min<size_t>(n, ctx->lane_chunk);
    const size_t lanes_padded = (lanes + 63) / 64 * 64;
    if ((e = acquire_scratch(S, lanes_padded * kAtabWordsPerLane * sizeof(uint32_t), s)) != hipSuccess)
      return hip_fail(e);
  }
  // a row launch is one chunk (n <= kRowMaxCap)
  RowSlot slot;
  uint32_t slot_k = 0;
  if (row && (e = row_slot_acquire(ctx, D, s, d_bitmap != nullptr, slot, slot_k)) != hipSuccess) return hip_fail(e);
  // the quad kernel of an armed host batch (one launch) tags its 16-signature
  // slices (as enqueue_verify_keyed's)
  const bool qtag = ctx->quad_poll && !sr && form == kFormQuad && d_bitmap && D.tag_arm && n <= kChunk;
  if (qtag) {
    slot = RowSlot{};
    slot.tagged = D.tag_arm;
    slot.seq = D.tag_seq;
    D.tag_used = true;
    D.tag_width = 16;
  }
  D.timing.harvest(ctx->stats, D.device_ms, D.timed_calls, false);
  Timing::Pair tp;
  const bool timed = ctx->timing_every && D.timing_seq++ % ctx->timing_every == 0;
  if (timed && (e = D.timing.begin(tp, s)) != hipSuccess) return hip_fail(e);
  const size_t chunk = lane ? ctx->lane_chunk : kChunk;
  for (size_t c = 0; c < n; c += chunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(chunk, n - c);
    if (sr)
      e = launch_verify_sr25519(cn, d_pk + 32 * c, d_sig + 64 * c, d_msg, d_off + c, D.d_btab,
                                static_cast<uint32_t*>(S.buf.p), D.d_srprog, ctx->sr_nops,
                                d_valid ? d_valid + c : nullptr, d_bitmap ? d_bitmap + c / 64 : nullptr, kflags, s);
    else
      e = launch_verify(mode, cn, d_pk + 32 * c, d_sig + 64 * c, d_msg, d_off + c, D.d_btab,
                        static_cast<uint32_t*>(S.buf.p), d_valid ? d_valid + c : nullptr,
                        d_bitmap ? d_bitmap + c / 64 : nullptr, kflags, s, sb, row || qtag ? &slot : nullptr);
    if (e == hipSuccess && row) e = row_slot_release(ctx, D, s, slot_k);
    if (e != hipSuccess) {
      D.timing.abandon(tp);
      return hip_fail(e);
    }
    ctx->stats.kernel_launches++;
    D.launches++;
  }
  if (lane && (e = release_scratch(S, s)) != hipSuccess) return hip_fail(e);
  if (timed && (e = D.timing.end(tp, s)) != hipSuccess) return hip_fail(e);
  ctx->stats.calls++;
  ctx->stats.signatures += n;
  D.calls++;
  D.signatures += n;
  return CMTV_OK;
}

// keys per comb-build launch (prefix-product scratch = 160 KiB per key)
constexpr uint32_t kCombKeyChunk = 256;

static int enqueue_verify_keyed(cmtv_ctx* ctx, CmtvDev& D, const cmtv_keyset::PerDev& K, size_t n_keys, size_t n,
                                const uint32_t* d_idx, const uint8_t* d_sig, const uint8_t* d_msg,
                                const uint32_t* d_off, uint32_t mode, uint8_t* d_valid, uint64_t* d_bitmap,
                                hipStream_t s, Scratch* scr = nullptr, const SbFuse* sb = nullptr,
                                uint32_t min_waves = 0) {
  if (n == 0) return CMTV_OK;
  if (!min_waves) min_waves = ctx->keyed_batch_min_waves;  // a masked bulk lane holds fewer
  Scratch& S = scr ? *scr : D.scratch;
  if (sb && !keyed_fuse_ok(ctx, n)) return CMTV_EINVAL;
  if (!d_idx && !sb) return CMTV_EINVAL;  // identity keys only in the one-launch fused forms
  if (fault_hit(ctx) || D.inject_fault) return CMTV_EHIP;
  const uint32_t form = keyed_form(ctx, n);
  // lane launches: KB signatures per lane sharing one inversion while that
  // still gives two waves per SIMD (k_verify_keyed_batch; ZIP-215 by coset)
  const bool batch = form == kKeyedLane;
  // batched launches of kKeyedBatchChunk = 2^20 signatures: one full round
  // of 2,048 waves at KB = 8 (equal launches of 1.07M measured 53.9 ms for
  // configs[2]'s 15M against 37.8 ms: 2,093 waves start a second, nearly
  // empty round)
  const size_t chunk = batch ? kKeyedBatchChunk : kChunk;
  auto kb_for = [&](size_t cn) -> uint32_t {  // 4 or 8 (the instantiated forms), else 1
    // the widest KB that still launches keyed_batch_min_waves waves (the last
    // one may be partial: a commit-aligned 1,048,500-signature chunk takes KB
    // = 8 in 2,048 waves)
    uint32_t kb = 1;
    while (kb < 8 && cn > ((size_t)min_waves - 1) * 64 * (kb * 2)) kb *= 2;
    return batch && kb >= 4 ? kb : 1;
  };
  hipError_t e;
  const uint32_t kb0 = kb_for(std::min(chunk, n));
  if (kb0 > 1) {
    const size_t lanes = (std::min(chunk, n) + 64 * kb0 - 1) / (64 * kb0) * 64;
    if ((e = acquire_scratch(S, lanes * kb0 * kKeyedBatchScratchWordsPerSig * sizeof(uint32_t), s)) != hipSuccess)
      return hip_fail(e);
  }
  // the keyed row kernel: one chunk, one slot of the bitmap ring
  const bool krow = form == kKeyedRow;
  RowSlot slot;
  uint32_t slot_k = 0;
  if (krow && (e = row_slot_acquire(ctx, D, s, d_bitmap != nullptr, slot, slot_k)) != hipSuccess)
    return hip_fail(e);
  // the keyed quad kernel of an armed host batch (one launch) tags its
  // 16-signature slices instead of writing the bitmap: the call polls them
  // (wait_row_tags) rather than wait for the stream
  RowSlot qtags;
  const bool qtag = ctx->quad_poll && form == kKeyedQuad && d_bitmap && D.tag_arm && n <= chunk;
  if (qtag) {
    qtags.tagged = D.tag_arm;
    qtags.seq = D.tag_seq;
    D.tag_used = true;
    D.tag_width = 16;
  }
  D.timing.harvest(ctx->stats, D.device_ms, D.timed_calls, false);
  Timing::Pair tp;
  const bool timed = ctx->timing_every && D.timing_seq++ % ctx->timing_every == 0;
  if (timed && (e = D.timing.begin(tp, s)) != hipSuccess) return hip_fail(e);
  for (size_t c = 0; c < n; c += chunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(chunk, n - c);
    // a chunk never needs more scratch than the first (kb and lanes shrink together)
    const uint32_t kb = kb0 > 1 ? kb_for(cn) : 1;
    e = launch_verify_keyed(mode, cn, (uint32_t)n_keys, d_idx ? d_idx + c : nullptr, d_sig + 64 * c, d_msg,
                            d_off + c, K.d_pk, K.d_ok, K.d_tab, d_valid ? d_valid + c : nullptr,
                            d_bitmap ? d_bitmap + c / 64 : nullptr, form, ctx->keyed_wait, D.d_diag, kb,
                            static_cast<uint32_t*>(S.buf.p), form == kKeyedLane ? K.d_wide : nullptr, D.d_btab, s,
                            krow ? &slot : qtag ? &qtags : nullptr, sb);
    if (e == hipSuccess && krow) e = row_slot_release(ctx, D, s, slot_k);
    if (e != hipSuccess) {
      D.timing.abandon(tp);
      return hip_fail(e);
    }
    ctx->stats.kernel_launches++;
    ctx->stats.keyed_launches++;
    D.launches++;
  }
  if (kb0 > 1 && (e = release_scratch(S, s)) != hipSuccess) return hip_fail(e);
  if (timed && (e = D.timing.end(tp, s)) != hipSuccess) return hip_fail(e);
  ctx->stats.calls++;
  ctx->stats.signatures += n;
  D.calls++;
  D.signatures += n;
  return CMTV_OK;
}

// ---------------------------------------------------------------- sharding

// Waits up to ctx->rccl_drain_ms for the streams of devices dev[0..G);
// false if one still has work queued (a collective that cannot complete).
static bool drain_bounded(cmtv_ctx* ctx, const size_t* dev, size_t G) {
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(ctx->rccl_drain_ms);
  for (size_t g = 0; g < G; g++) {
    CmtvDev& D = ctx->devs[dev[g]];
    (void)hipSetDevice(D.ordinal);
    for (;;) {
      const hipError_t q = hipStreamQuery(D.stream);
      if (q != hipErrorNotReady) break;  // done (or failed: nothing left to wait for)
      if (std::chrono::steady_clock::now() > t_end) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  }
  (void)hipGetLastError();
  return true;
}

// Releases every device's communicator; abort = ncclCommAbort where the
// library has it (ends collectives stuck on their peers), else CommDestroy.
static void drop_comms(cmtv_ctx* ctx, bool abort) {
  const Rccl& R = rccl(ctx->rccl_lib);
  for (auto& D : ctx->devs) {
    if (D.comm && R.ok) {
      (void)hipSetDevice(D.ordinal);
      if (abort && R.CommAbort)
        (void)R.CommAbort(D.comm);
      else
        (void)R.CommDestroy(D.comm);
    }
    D.comm = nullptr;
  }
}

// Bitmap all-gather over the devices dev[0..G): the one at position g holds
// its shard in words [g W, (g+1) W) of bufs[g] (G x W words each); afterwards
// every bufs[g] holds all shards. RCCL all-gather in place when the context
// has a communicator (then dev must be ctx->live, the communicator's ranks in
// order), else peer copies (a context over a repeated device ordinal).
// Enqueued on the device streams.
static int gather_bitmaps(cmtv_ctx* ctx, const size_t* dev, size_t G, size_t W, uint64_t* const* bufs) {
  // one device: nothing to exchange, unless CMTV_FORCE_RCCL gave it a
  // one-rank communicator (the RCCL path exercised on a one-GPU box)
  if (G <= 1 && !ctx->rccl) return CMTV_OK;
  ctx->stats.gathers++;
  if (ctx->rccl) {
    const Rccl& R = rccl(ctx->rccl_lib);
    int bad = R.GroupStart() != 0;
    for (size_t g = 0; g < G && !bad; g++) {
      CmtvDev& D = ctx->devs[dev[g]];
      (void)hipSetDevice(D.ordinal);
      bad |= R.AllGather(bufs[g] + g * W, bufs[g], W, kNcclUint64, D.comm, D.stream) != 0;
    }
    bad |= R.GroupEnd() != 0;
    if (!bad) return CMTV_OK;
    // RCCL refused the gather (a node whose xGMI / RCCL setup fails at run
    // time). Some ranks' collectives may already be enqueued (RCCL launches
    // each rank's kernel at GroupEnd): they wait for peers that never come,
    // and anything queued behind them would hang. So the communicators go
    // (aborted when a stream does not drain within rccl_drain_ms, which ends
    // a stuck collective), the context never builds one again, and only a
    // gather whose streams drained falls back to peer copies below -- this one
    // and every later one; CMTV_NO_RCCL_FALLBACK=1 reports CMTV_ERCCL instead.
    ctx->stats.rccl_failures++;
    const bool drained = drain_bounded(ctx, dev, G);
    drop_comms(ctx, !drained);
    ctx->rccl_broken = true;
    ctx->rccl = false;
    ctx->stats.rccl = 0;
    if (!drained) {
      // an aborted collective leaves its stream in an error state: wait once
      // more (bounded) so a later call does not queue behind it
      (void)drain_bounded(ctx, dev, G);
      return CMTV_ERCCL;
    }
    if (ctx->no_rccl_fallback) return CMTV_ERCCL;
  }
  hipError_t e;
  for (size_t h = 0; h < G; h++) {
    CmtvDev& H = ctx->devs[dev[h]];
    (void)hipSetDevice(H.ordinal);
    if ((e = hipEventRecord(H.done, H.stream)) != hipSuccess) return hip_fail(e);
  }
  for (size_t g = 0; g < G; g++) {
    CmtvDev& D = ctx->devs[dev[g]];
    (void)hipSetDevice(D.ordinal);
    for (size_t h = 0; h < G; h++) {
      if (h == g) continue;
      CmtvDev& H = ctx->devs[dev[h]];
      if ((e = hipStreamWaitEvent(D.stream, H.done, 0)) != hipSuccess) return hip_fail(e);
      if ((e = hipMemcpyPeerAsync(bufs[g] + h * W, D.ordinal, bufs[h] + h * W, H.ordinal, W * 8, D.stream)) !=
          hipSuccess)
        return hip_fail(e);
    }
  }
  // the copies read other devices' buffers: finish them before those
  // devices' next kernels may write
  for (size_t g = 0; g < G; g++) {
    CmtvDev& D = ctx->devs[dev[g]];
    (void)hipSetDevice(D.ordinal);
    if ((e = hipStreamSynchronize(D.stream)) != hipSuccess) return hip_fail(e);
  }
  return CMTV_OK;
}

// A batch in host memory: generic (pk rows), registered keys (key_idx into
// ks) or sr25519; messages either host-encoded (msg) or written on the
// device from per-commit CanonicalVote templates (signbytes.h).
struct HostBatch {
  size_t n = 0;
  uint32_t mode = 0;
  const uint8_t* pk = nullptr;
  const cmtv_keyset* ks = nullptr;
  const uint32_t* key_idx = nullptr;
  const uint8_t* sig = nullptr;
  const uint32_t* msg_off = nullptr;
  uint32_t msg_bound = 0;  // templated with msg_off null: every message is at most this long
  const uint8_t* msg = nullptr;
  const SbTemplate* tmpls = nullptr;
  size_t n_tmpls = 0;
  const uint8_t* blob = nullptr;
  size_t blob_len = 0;
  const uint32_t* tidx = nullptr;
  const uint8_t* tflag = nullptr;
  const int64_t* sec = nullptr;
  const int32_t* nanos = nullptr;
  // a speculative launch (commit.cpp's speculative VerifyCommit): run once
  // the batch's kernels are enqueued, before the call waits for them; its
  // answer goes to *between_ok (the caller discards the verdicts on false)
  const std::function<bool()>* between = nullptr;
  bool* between_ok = nullptr;
  void after_launch() const {
    if (between) *between_ok = (*between)();
  }
};

// Stage rows [a, b) of B on device g and enqueue sign-bytes (templated) and
// verification; verdict bytes to D.d_out (when want_valid), bitmap words to
// `bitmap` (device memory of D).
static int enqueue_shard(cmtv_ctx* ctx, size_t g, const HostBatch& B, size_t a, size_t b, bool want_valid,
                         uint64_t* bitmap, size_t& o_valid_out, bool zero_copy = false) {
  CmtvDev& D = ctx->devs[g];
  const size_t m = b - a;
  const bool keyed = B.ks != nullptr, tpl = B.msg == nullptr;
  // no offsets (verify_templated_locked: the fused small-batch path only):
  // sized by the bound, never written
  const bool no_off = tpl && !B.msg_off;
  const size_t mb = no_off ? (size_t)B.msg_bound * m : (size_t)B.msg_off[b] - B.msg_off[a];
  const size_t key_bytes = keyed ? 4 * m : 32 * m;
  // signatures first: an early-staged commit's (stage_sigs_early_locked) are
  // already there, on their way to the device
  const size_t o_sig = 0, o_key = align_up(64 * m, 256), o_off = align_up(o_key + key_bytes, 256);
  size_t o_tidx = 0, o_flag = 0, o_sec = 0, o_nanos = 0, o_tmpl = 0, o_blob = 0, in_bytes, o_msg, dev_bytes;
  const size_t tb = B.n_tmpls * sizeof(SbTemplate);
  if (tpl) {
    o_tidx = align_up(o_off + 4 * (m + 1), 256);
    o_flag = align_up(o_tidx + 4 * m, 256);
    o_sec = align_up(o_flag + m, 256);
    o_nanos = align_up(o_sec + 8 * m, 256);
    o_tmpl = align_up(o_nanos + 4 * m, 256);
    o_blob = align_up(o_tmpl + tb, 256);
    in_bytes = align_up(o_blob + B.blob_len + 16, 256);
    o_msg = in_bytes;  // device only: k_sign_bytes writes the messages here
    dev_bytes = align_up(o_msg + mb + 16, 256);
  } else {
    o_msg = align_up(o_off + 4 * (m + 1), 256);
    in_bytes = align_up(o_msg + mb + 16, 256);
    dev_bytes = in_bytes;
  }
  const size_t o_valid = 0, out_bytes = align_up(std::max<size_t>(m, 1), 256);
  o_valid_out = o_valid;
  hipError_t e;
  const uint64_t t_stage = phase_now(ctx);
  (void)hipSetDevice(D.ordinal);
  // message lengths first: they decide the fused / zero-copy forms
  const uint32_t base = no_off ? 0u : B.msg_off[a];
  uint32_t max_len = no_off ? B.msg_bound : 0u;
  if (!no_off)
    for (size_t i = 0; i < m; i++) max_len = std::max(max_len, B.msg_off[a + i + 1] - B.msg_off[a + i]);
  // templated sign-bytes written by the verify kernel's helper wave (no
  // k_sign_bytes launch) when the batch runs a split kernel and every
  // message fits the helper's LDS slot; CMTV_NO_SB_FUSE turns it off
  const bool fuse = tpl && ctx->sb_fuse && max_len <= kSbFuseMaxMsg && (keyed ? keyed_fuse_ok(ctx, m) : fuse_ok(ctx, m));
  // a fused small batch reads its staging in mapped host memory directly
  // (CMTV_NO_ZC_IN turns it off), and so does a small plain host-API batch
  // whose messages fit the same bound (keys, signatures and messages; no
  // sign-bytes kernel writes into the staging then; CMTV_ZC_HOST_IN=0 copies
  // it). Measured on MI355X (round 4, profiles/r04_zc_host_ab.txt): host API
  // 150 0.116 -> 0.109 ms, 4,096 0.284 -> 0.269, 10,000 0.343 -> 0.326 ms.
  // Registered-key batches copy it (their signatures are early-staged past
  // the keyed row band): reading all of it in place was measured no faster
  // at 150 (p50 0.0525 vs 0.0523-0.0534 ms) and slower at 10k (0.144-0.148
  // vs 0.136-0.137 ms, kernel 0.089-0.093 vs 0.078 ms; round 5,
  // profiles/r05_zc_keyed_ab.txt), and that option was retired.
  // the signatures (and keys) staged ahead of the plan: the same bytes are
  // already in h_in (and on their way to d_in on this stream), unless a
  // buffer must grow; a batch that has them reads HBM, not its staging in place
  const bool early = D.early_src && D.early_src == B.sig + 64 * a && m <= D.early_n && in_bytes <= D.h_in.cap &&
                     dev_bytes <= D.d_in.cap;
  const bool early_pk = early && !keyed && D.early_pk && D.early_pk == B.pk + 32 * a && m == D.early_n;
  D.early_src = D.early_pk = nullptr;
  const bool zc = !early && (!keyed || ctx->keyed_zc || (ctx->bulk_now && ctx->load_zc)) && zero_copy && ctx->zc_in &&
                  (fuse || (!tpl && ctx->zc_host_in && max_len <= kSbFuseMaxMsg));
  // split: the early-staged signatures (and keys) in HBM, the rest -- the
  // fused helper's templates, flags and timestamps, ~17 bytes a signature --
  // read in place from mapped memory, so the launch waits for no second copy.
  // Measured on MI355X (tools/early_ab.sh, three alternating rounds):
  // verify_commit_10k_keyset p50 0.1435-0.1443 -> 0.1350-0.1359 ms (kernel
  // +3 us: its hash helper reads the fields over PCIe), verify_commit_10k
  // 0.293-0.303 -> 0.289-0.294 ms.
  const bool split = early && zero_copy && ctx->zc_in && fuse && (keyed || early_pk);
  HostBuf& HB = (zc || split) ? D.h_zin : D.h_in;
  if ((e = HB.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if (!zc && (e = D.d_in.ensure(dev_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = D.d_out.ensure(out_bytes)) != hipSuccess) return hip_fail(e);
  auto* hin = static_cast<uint8_t*>(HB.p);
  // a null key_idx (registered keys) means signature i is by key i, a null
  // tidx that every signature uses template 0: the fused kernels take them
  // as null, anything else gets the arrays written out
  const bool null_kidx = keyed && !B.key_idx && fuse, null_tidx = tpl && !B.tidx && fuse;
  if (keyed) {
    if (B.key_idx)
      std::memcpy(hin + o_key, B.key_idx + a, 4 * m);
    else if (!null_kidx)
      for (size_t i = 0; i < m; i++) reinterpret_cast<uint32_t*>(hin + o_key)[i] = (uint32_t)(a + i);
  } else if (!early_pk) {
    std::memcpy(hin + o_key, B.pk + 32 * a, 32 * m);
  }
  // zero-copy signatures already in the caller's cmtv_alloc_pinned memory are
  // read from there (no host copy)
  const bool sig_in_place = zc && pinned_holds_locked(ctx, B.sig + 64 * a, 64 * m);
  if (!early && !sig_in_place) std::memcpy(hin + o_sig, B.sig + 64 * a, 64 * m);
  if (no_off && !fuse) return CMTV_EINVAL;  // verify_templated_locked derives offsets for every other form
  auto* hoff = reinterpret_cast<uint32_t*>(hin + o_off);
  if (!no_off)
    for (size_t i = 0; i <= m; i++) hoff[i] = B.msg_off[a + i] - base;
  if (tpl) {
    if (B.tidx)
      std::memcpy(hin + o_tidx, B.tidx + a, 4 * m);
    else if (!null_tidx)
      std::memset(hin + o_tidx, 0, 4 * m);
    std::memcpy(hin + o_flag, B.tflag + a, m);
    std::memcpy(hin + o_sec, B.sec + a, 8 * m);
    std::memcpy(hin + o_nanos, B.nanos + a, 4 * m);
    std::memcpy(hin + o_tmpl, B.tmpls, tb);
    if (B.blob_len) std::memcpy(hin + o_blob, B.blob, B.blob_len);
  } else {
    if (mb) std::memcpy(hin + o_msg, B.msg + base, mb);
    std::memset(hin + o_msg + mb, 0, 16);
  }
  phase_add(ctx, kPhStage, t_stage);
  const uint64_t t_launch = phase_now(ctx);
  uint8_t* din = static_cast<uint8_t*>(D.d_in.p);
  uint8_t* dmsg = din + o_msg;  // the templated sign-bytes, written by k_sign_bytes
  auto* dout = static_cast<uint8_t*>(D.d_out.p);
  // where the kernel reads the signatures and (generic) keys: HBM unless
  // the whole staging is read in place
  uint8_t* dsig = din + o_sig;
  uint8_t* dkey = din + o_key;
  if (zc || split) {
    void* p = nullptr;
    if ((e = hipHostGetDevicePointer(&p, HB.p, 0)) != hipSuccess) return hip_fail(e);
    din = static_cast<uint8_t*>(p);
    dmsg = din + o_msg;
    if (zc) dsig = din + o_sig;
    if (sig_in_place) {
      void* q = nullptr;
      if ((e = hipHostGetDevicePointer(&q, const_cast<uint8_t*>(B.sig + 64 * a), 0)) != hipSuccess) return hip_fail(e);
      dsig = static_cast<uint8_t*>(q);
    }
    if (zc || keyed) dkey = din + o_key;  // key indices (keyed) are in the mapped staging
  } else {
    const size_t from = early_pk ? o_off : early ? o_key : 0;  // what the early copy did not carry
    if ((e = hipMemcpyAsync(din + from, hin + from, in_bytes - from, hipMemcpyHostToDevice, D.stream)) != hipSuccess)
      return hip_fail(e);
  }
  SbFuse sb;
  if (fuse) {
    sb.tmpls = din + o_tmpl;
    sb.blob = din + o_blob;
    sb.tidx = null_tidx ? nullptr : reinterpret_cast<uint32_t*>(din + o_tidx);
    sb.flag = din + o_flag;
    sb.sec = reinterpret_cast<int64_t*>(din + o_sec);
    sb.nanos = reinterpret_cast<int32_t*>(din + o_nanos);
    ctx->stats.fused_sign_bytes++;
  } else if (tpl) {
    // k_sign_bytes also writes the 16 zero bytes after the last message
    if ((e = launch_sign_bytes((uint32_t)m, din + o_tmpl, din + o_blob, reinterpret_cast<uint32_t*>(din + o_tidx),
                               din + o_flag, reinterpret_cast<int64_t*>(din + o_sec),
                               reinterpret_cast<int32_t*>(din + o_nanos), reinterpret_cast<uint32_t*>(din + o_off),
                               dmsg, D.stream)) != hipSuccess)
      return hip_fail(e);
  }
  uint8_t* dv = want_valid ? dout + o_valid : nullptr;
  int rc;
  if (keyed)
    rc = enqueue_verify_keyed(ctx, D, B.ks->dev[g], B.ks->n, m,
                              null_kidx ? nullptr : reinterpret_cast<uint32_t*>(dkey), dsig,
                              tpl ? dmsg : din + o_msg, reinterpret_cast<uint32_t*>(din + o_off), B.mode, dv, bitmap,
                              D.stream, nullptr, fuse ? &sb : nullptr);
  else
    rc = enqueue_verify(ctx, D, m, dkey, dsig, din + o_msg, reinterpret_cast<uint32_t*>(din + o_off), B.mode, dv,
                        bitmap, D.stream, fuse ? &sb : nullptr);
  phase_add(ctx, kPhLaunch, t_launch);
  return rc;
}

// Verdicts of a host batch, sharded over the context's live devices. Caller
// holds the lock. On a device's HIP error *bad_dev names it.
// Wait for a tagged row launch (CmtvDev::tag_used) of n signatures on device
// D: poll the entries until each carries the call's tag, asking the stream
// every 256 polls so that an error ends the wait; a launch that finished with
// an entry untagged (which cannot happen) is an error, not a hang.
// A small host batch's wait for its stream: hipStreamSynchronize, or with
// spin_wait (CMTV_SPIN_WAIT=1, A/B knob) a busy poll of hipStreamQuery that
// keeps the calling thread on its CPU
static hipError_t wait_stream(const cmtv_ctx* ctx, hipStream_t s) {
  if (!ctx->spin_wait) return hipStreamSynchronize(s);
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q != hipErrorNotReady) return q;
  }
}

static hipError_t wait_row_tags(CmtvDev& D, size_t n) {
  const uint64_t* e = static_cast<const uint64_t*>(D.h_tags.p);
  const size_t n32 = (n + D.tag_width - 1) / D.tag_width;  // entries
  size_t j = 0;
  auto scan = [&] {
    while (j < n32 && (uint32_t)(__atomic_load_n(e + j, __ATOMIC_ACQUIRE) >> 32) == D.tag_seq) j++;
    return j == n32;
  };
  for (uint32_t spin = 1;; spin++) {
    if (scan()) return hipSuccess;
    if ((spin & 255) == 0) {
      const hipError_t q = hipStreamQuery(D.stream);
      if (q == hipSuccess) return scan() ? hipSuccess : hipErrorLaunchFailure;
      if (q != hipErrorNotReady) return q;
    }
  }
}

static int run_host_batch_(cmtv_ctx* ctx, const HostBatch& B, uint8_t* out_valid, uint64_t* out_bitmap,
                           long* bad_dev) {
  const size_t n = B.n;
  if (n == 0) return CMTV_OK;
  const std::vector<size_t>& live = ctx->live;
  if (live.empty()) return CMTV_ENODEV;
  const ShardPlan P = plan_shards(n, live.size(), ctx->shard_min);
  const size_t words = (n + 63) / 64;
  hipError_t e;
  const size_t d0 = live[0];
  if (P.G == 1 && n <= ctx->zc_max) {
    // one device, a small batch: the verify kernel writes the bitmap into
    // mapped host memory, so the call is H2D + (sign-bytes) + verify + sync
    CmtvDev& D = ctx->devs[d0];
    *bad_dev = (long)d0;
    (void)hipSetDevice(D.ordinal);
    // the previous polled launch read h_zin: it must be done before the
    // staging below overwrites it
    if ((e = settle_polled(D)) != hipSuccess) return hip_fail(e);
    if ((e = D.h_zc.ensure(8 * words)) != hipSuccess) return hip_fail(e);
    void* dzc = nullptr;
    if ((e = hipHostGetDevicePointer(&dzc, D.h_zc.p, 0)) != hipSuccess) return hip_fail(e);
    // a row launch tags its bitmap words (kernels.h RowSlot; CMTV_HOST_POLL=0:
    // it writes the bitmap and the call waits for the stream)
    if (ctx->host_poll && !D.d_tags) {
      void* dt = nullptr;
      if ((e = D.h_tags.ensure(8 * kTagEntries)) != hipSuccess) return hip_fail(e);
      std::memset(D.h_tags.p, 0, 8 * kTagEntries);
      if ((e = hipHostGetDevicePointer(&dt, D.h_tags.p, 0)) != hipSuccess) return hip_fail(e);
      D.d_tags = static_cast<uint64_t*>(dt);
    }
    // ... but not beside a pipeline call (bulk_now): polled under a configs[2]
    // load the 150-validator call's p99 was 1.05-1.11 ms against 0.148 ms
    // waiting for the stream (round 6, tools/gpu_r6o.sh)
    const bool poll = ctx->host_poll && !(ctx->bulk_now && ctx->load_nopoll);
    if (poll && ++D.tag_seq == 0) D.tag_seq = 1;
    D.tag_arm = poll ? D.d_tags : nullptr;
    D.tag_used = false;
    size_t o_valid = 0;
    // CMTV_CALL_TRACE: the device time of this call's work, between two events
    if (ctx->call_trace) {
      if (!ctx->trace_ev[0]) {
        (void)hipEventCreate(&ctx->trace_ev[0]);
        (void)hipEventCreate(&ctx->trace_ev[1]);
      }
      (void)hipEventRecord(ctx->trace_ev[0], D.stream);
    }
    const int rc = enqueue_shard(ctx, d0, B, 0, n, false, static_cast<uint64_t*>(dzc), o_valid, true);
    if (ctx->call_trace) (void)hipEventRecord(ctx->trace_ev[1], D.stream);
    D.tag_arm = nullptr;
    if (rc != CMTV_OK) return rc;
    B.after_launch();
    if (D.tag_used) {  // settled by the next call (settle_polled)
      if (!D.poll_ev && (e = hipEventCreateWithFlags(&D.poll_ev, hipEventDisableTiming)) != hipSuccess)
        return hip_fail(e);
      if ((e = hipEventRecord(D.poll_ev, D.stream)) != hipSuccess) return hip_fail(e);
      D.poll_pending = true;
    }
    const uint64_t t_wait = phase_now(ctx);
    if (ctx->call_trace) ctx->trace_launch = call_trace_now();
    if ((e = D.tag_used ? wait_row_tags(D, n) : wait_stream(ctx, D.stream)) != hipSuccess) return hip_fail(e);
    if (ctx->call_trace) {
      ctx->trace_wait = call_trace_now();
      float ms = 0;
      if (!D.tag_used && hipEventElapsedTime(&ms, ctx->trace_ev[0], ctx->trace_ev[1]) == hipSuccess)
        ctx->trace_dev_ns = (uint64_t)(ms * 1e6f);
      else
        ctx->trace_dev_ns = 0;
    }
    uint64_t* bm = static_cast<uint64_t*>(D.h_zc.p);
    if (D.tag_used) {
      ctx->stats.polled_calls++;
      const uint64_t* tg = static_cast<const uint64_t*>(D.h_tags.p);
      if (D.tag_width == 32) {
        const size_t n32 = (n + 31) / 32;
        for (size_t w = 0; w < words; w++)
          bm[w] = (tg[2 * w] & 0xFFFFFFFFull) | (2 * w + 1 < n32 ? (tg[2 * w + 1] & 0xFFFFFFFFull) << 32 : 0);
      } else {
        const size_t n16 = (n + 15) / 16;
        for (size_t w = 0; w < words; w++) {
          uint64_t x = 0;
          for (size_t k = 0; k < 4 && 4 * w + k < n16; k++) x |= (tg[4 * w + k] & 0xFFFFull) << (16 * k);
          bm[w] = x;
        }
      }
    }
    phase_add(ctx, kPhWait, t_wait);
    const uint64_t t_post = phase_now(ctx);
    if ((long)d0 == ctx->fault_sync_dev) {  // CMTV_FAULT_SYNC_DEV (see below)
      ctx->stats.faults_injected++;
      return CMTV_EHIP;
    }
    *bad_dev = -1;
    harvest(ctx, false);
    (void)hipSetDevice(D.ordinal);
    // bits past n of the last word are not written by every kernel
    if (n & 63) bm[words - 1] &= (1ull << (n & 63)) - 1;
    uint64_t valid_count = 0;
    for (size_t w = 0; w < words; w++) valid_count += (uint64_t)__builtin_popcountll(bm[w]);
    ctx->stats.invalid += n - valid_count;
    if (out_bitmap) std::memcpy(out_bitmap, bm, 8 * words);
    if (out_valid)
      for (size_t i = 0; i < n; i++) out_valid[i] = (uint8_t)((bm[i >> 6] >> (i & 63)) & 1);
    phase_add(ctx, kPhPost, t_post);
    return CMTV_OK;
  }
  // devices in the gather: the shards' devices, or with RCCL every rank of
  // the communicator (a rank without a shard contributes zero words)
  const size_t GG = P.G == 1 ? 1 : (ctx->rccl ? live.size() : P.G);
  uint64_t* bufs[kMaxDevices];
  for (size_t g = 0; g < GG; g++) {
    CmtvDev& D = ctx->devs[live[g]];
    *bad_dev = (long)live[g];
    (void)hipSetDevice(D.ordinal);
    if ((e = D.d_all.ensure(8 * std::max<size_t>(GG * P.W, 1))) != hipSuccess) return hip_fail(e);
    bufs[g] = static_cast<uint64_t*>(D.d_all.p);
  }
  size_t o_valid = 0;
  for (size_t g = 0; g < GG; g++) {
    const size_t a = P.lo(g, n), b = P.hi(g, n);
    *bad_dev = (long)live[g];
    if (a == b) {
      // an empty shard still takes part in the gather
      (void)hipSetDevice(ctx->devs[live[g]].ordinal);
      if ((e = hipMemsetAsync(bufs[g] + g * P.W, 0, 8 * P.W, ctx->devs[live[g]].stream)) != hipSuccess)
        return hip_fail(e);
      continue;
    }
    const int rc = enqueue_shard(ctx, live[g], B, a, b, P.G == 1, bufs[g] + g * P.W, o_valid);
    if (rc != CMTV_OK) return rc;
  }
  *bad_dev = -1;
  B.after_launch();
  if (P.G > 1) {
    ctx->stats.sharded_calls++;
    const int rc = gather_bitmaps(ctx, live.data(), GG, P.W, bufs);
    if (rc != CMTV_OK) return rc;
  }
  // results from the first live device: verdict bytes + bitmap (one device)
  // or the gathered bitmap (several)
  CmtvDev& D0 = ctx->devs[d0];
  (void)hipSetDevice(D0.ordinal);
  const size_t o_bm = 0, o_v = align_up(8 * words, 256);
  const size_t out_bytes = P.G == 1 ? align_up(o_v + n, 256) : 8 * words;
  if ((e = D0.h_out.ensure(out_bytes)) != hipSuccess) return hip_fail(e);
  auto* hout = static_cast<uint8_t*>(D0.h_out.p);
  if ((e = hipMemcpyAsync(hout + o_bm, bufs[0], 8 * words, hipMemcpyDeviceToHost, D0.stream)) != hipSuccess)
    return hip_fail(e);
  if (P.G == 1 &&
      (e = hipMemcpyAsync(hout + o_v, static_cast<uint8_t*>(D0.d_out.p) + o_valid, n, hipMemcpyDeviceToHost,
                          D0.stream)) != hipSuccess)
    return hip_fail(e);
  const uint64_t t_wait = phase_now(ctx);
  for (size_t g = 0; g < GG; g++) {
    *bad_dev = (long)live[g];
    (void)hipSetDevice(ctx->devs[live[g]].ordinal);
    if ((e = hipStreamSynchronize(ctx->devs[live[g]].stream)) != hipSuccess) return hip_fail(e);
    // CMTV_FAULT_SYNC_DEV: this device's work "failed" after its launch
    if ((long)live[g] == ctx->fault_sync_dev) {
      ctx->stats.faults_injected++;
      return CMTV_EHIP;
    }
  }
  *bad_dev = -1;
  phase_add(ctx, kPhWait, t_wait);
  const uint64_t t_post = phase_now(ctx);
  (void)hipSetDevice(D0.ordinal);
  harvest(ctx, false);
  (void)hipSetDevice(D0.ordinal);
  uint64_t* bm = reinterpret_cast<uint64_t*>(hout + o_bm);
  // bits past n of the last word are not written by every kernel
  if (n & 63) bm[words - 1] &= (1ull << (n & 63)) - 1;
  uint64_t valid_count = 0;
  for (size_t w = 0; w < words; w++) valid_count += (uint64_t)__builtin_popcountll(bm[w]);
  ctx->stats.invalid += n - valid_count;
  if (out_bitmap) std::memcpy(out_bitmap, bm, 8 * words);
  if (out_valid) {
    if (P.G == 1) {
      std::memcpy(out_valid, hout + o_v, n);
    } else {
      for (size_t i = 0; i < n; i++) out_valid[i] = (uint8_t)((bm[i >> 6] >> (i & 63)) & 1);
    }
  }
  phase_add(ctx, kPhPost, t_post);
  return CMTV_OK;
}

static void rebuild_comm(cmtv_ctx* ctx);

// Takes device d out of the context's rotation after a HIP error
// (per-GPU failure -> re-shard onto the remaining GPUs; the
// libs/fail/fail.go analogue is CMTV_FAULT_DEV). Its communicator rank goes
// too: the RCCL communicator is rebuilt over the survivors.
static void retire_device(cmtv_ctx* ctx, size_t d) {
  if (ctx->devs[d].failed) return;
  ctx->devs[d].failed = true;
  ctx->stats.device_failures++;
  ctx->live.erase(std::remove(ctx->live.begin(), ctx->live.end(), d), ctx->live.end());
  rebuild_comm(ctx);
}

static void drain(cmtv_ctx* ctx) {
  // work already enqueued for other shards still reads the pinned staging
  // the next call refills: drain it before returning or retrying
  for (auto& D : ctx->devs) {
    (void)hipSetDevice(D.ordinal);
    (void)hipStreamSynchronize(D.stream);
  }
  (void)hipGetLastError();
}

static int run_host_batch(cmtv_ctx* ctx, const HostBatch& B, uint8_t* out_valid, uint64_t* out_bitmap) {
  int rc = CMTV_OK;
  // every launch of this call is waited for before it returns (or drained)
  struct HostSync {
    cmtv_ctx* c;
    explicit HostSync(cmtv_ctx* x) : c(x) { c->host_sync = true; }
    ~HostSync() { c->host_sync = false; }
  } host_sync(ctx);
  // a device error retires that device and re-plans the batch over the
  // others, once per surviving device at most
  for (size_t attempt = 0; attempt < ctx->devs.size(); attempt++) {
    long bad = -1;
    rc = run_host_batch_(ctx, B, out_valid, out_bitmap, &bad);
    if (rc == CMTV_OK) break;
    drain(ctx);
    // only a device's own HIP error retires it (not CMTV_FAULT_AT, which
    // stands for a failure of the call, nor an allocation failure)
    const bool injected = ctx->fault_pending;
    ctx->fault_pending = false;
    if (rc != CMTV_EHIP || injected || bad < 0 || ctx->live.size() < 2) break;
    retire_device(ctx, (size_t)bad);
    ctx->stats.reshards++;
  }
  for (auto& D : ctx->devs) D.early_src = nullptr;  // used by this batch or never
  (void)hipSetDevice(ctx->devs[ctx->live.empty() ? 0 : ctx->live[0]].ordinal);
  return rc;
}

static const uint8_t kNoMessageBytes = 0;

static int verify_host_device(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                              const uint32_t* msg_off, uint32_t mode, uint8_t* out_valid, uint64_t* out_bitmap) {
  if (!msg) msg = &kNoMessageBytes;  // all messages empty (a null msg selects templated sign-bytes)
  HostBatch B;
  B.n = n;
  B.mode = mode;
  B.pk = pk;
  B.sig = sig;
  B.msg = msg;
  B.msg_off = msg_off;
  return run_host_batch(ctx, B, out_valid, out_bitmap);
}

bool cache_enabled(const cmtv_ctx* ctx) { return ctx->cache.cap != 0; }

int verify_host_locked(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                       const uint32_t* msg_off, uint32_t mode, uint8_t* out_valid, uint64_t* out_bitmap) {
  if (n == 0) return CMTV_OK;
  if (!ctx->cache.cap) return verify_host_device(ctx, n, pk, sig, msg, msg_off, mode, out_valid, out_bitmap);
  // cache lookups; the misses go to the device as one compacted batch
  std::vector<uint8_t> valid(n);
  std::vector<size_t> miss;
  std::vector<uint64_t> hs(n);
  std::vector<std::string> keys(n);
  for (size_t i = 0; i < n; i++) {
    VerdictCache::make_key(keys[i], mode, pk + 32 * i, sig + 64 * i, msg + msg_off[i], msg_off[i + 1] - msg_off[i]);
    hs[i] = ctx->cache.hash(keys[i]);
    const int v = ctx->cache.find(hs[i], keys[i]);
    if (v < 0)
      miss.push_back(i);
    else
      valid[i] = (uint8_t)v;
  }
  ctx->stats.cache_hits += n - miss.size();
  if (!miss.empty()) {
    const size_t m = miss.size();
    std::vector<uint8_t> mpk(32 * m), msg_(64 * m), mmsg, mv(m);
    std::vector<uint32_t> moff(m + 1, 0);
    for (size_t j = 0; j < m; j++) {
      const size_t i = miss[j];
      std::memcpy(&mpk[32 * j], pk + 32 * i, 32);
      std::memcpy(&msg_[64 * j], sig + 64 * i, 64);
      mmsg.insert(mmsg.end(), msg + msg_off[i], msg + msg_off[i + 1]);
      moff[j + 1] = (uint32_t)mmsg.size();
    }
    if (mmsg.empty()) mmsg.push_back(0);
    const int rc = verify_host_device(ctx, m, mpk.data(), msg_.data(), mmsg.data(), moff.data(), mode, mv.data(),
                                      nullptr);
    if (rc != CMTV_OK) return rc;
    for (size_t j = 0; j < m; j++) {
      const size_t i = miss[j];
      valid[i] = mv[j];
      ctx->cache.insert(hs[i], std::move(keys[i]), mv[j]);
    }
  }
  if (out_valid) std::memcpy(out_valid, valid.data(), n);
  if (out_bitmap) {
    const size_t words = (n + 63) / 64;
    for (size_t w = 0; w < words; w++) {
      uint64_t x = 0;
      for (size_t b = 0; b < 64 && 64 * w + b < n; b++) x |= (uint64_t)(valid[64 * w + b] & 1) << b;
      out_bitmap[w] = x;
    }
  }
  return CMTV_OK;
}

int verify_templated_locked(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint32_t* msg_off,
                            const void* tmpls, size_t n_tmpls, const uint8_t* blob, size_t blob_len,
                            const uint32_t* tidx, const uint8_t* commit_flag, const int64_t* sec,
                            const int32_t* nanos, uint32_t mode, uint8_t* out_valid, const cmtv_keyset* ks,
                            const uint32_t* key_idx, uint32_t msg_bound, const std::function<bool()>* between,
                            bool* between_ok) {
  // no offsets: the fused kernels of a small single-device batch build every
  // message from its template and never read them (enqueue_shard); any other
  // form gets them derived here, exactly as sb_msg_len gives them
  std::vector<uint32_t> off_v;
  if (!msg_off) {
    const bool fused_small = ctx->live.size() == 1 && n <= ctx->zc_max && ctx->sb_fuse && msg_bound <= kSbFuseMaxMsg &&
                             (ks ? keyed_fuse_ok(ctx, n) : fuse_ok(ctx, n));
    if (!fused_small) {
      off_v.resize(n + 1);
      uint64_t o = 0;
      const auto* tp = static_cast<const SbTemplate*>(tmpls);
      for (size_t i = 0; i < n; i++) {
        off_v[i] = (uint32_t)o;
        o += sb_msg_len(tp[tidx ? tidx[i] : 0], commit_flag[i] != 0, sec[i], nanos[i]);
      }
      if (o + 16 >= (1ull << 31)) return CMTV_EINVAL;
      off_v[n] = (uint32_t)o;
      msg_off = off_v.data();
    }
  }
  HostBatch B;
  B.n = n;
  B.mode = mode;
  B.pk = ks ? nullptr : pk;
  B.ks = ks;
  B.key_idx = key_idx;
  B.sig = sig;
  B.msg_off = msg_off;
  B.msg_bound = msg_bound;
  B.tmpls = static_cast<const SbTemplate*>(tmpls);
  B.n_tmpls = n_tmpls;
  B.blob = blob;
  B.blob_len = blob_len;
  B.tidx = tidx;
  B.tflag = commit_flag;
  B.between = between;
  B.between_ok = between_ok;
  B.sec = sec;
  B.nanos = nanos;
  return run_host_batch(ctx, B, out_valid, nullptr);
}

// A single-commit VerifyCommit on one device with registered keys spends
// ~25 us planning 10k signatures before its staging is copied: its
// signatures (the bulk of the staging) go to the device first, so their H2D
// copy overlaps the plan. Their bytes are only used if the batch that
// follows stages exactly those signatures on this device (enqueue_shard);
// otherwise they are overwritten unused.
int stage_sigs_early_locked(cmtv_ctx* ctx, const uint8_t* sigs, size_t n, const uint8_t* pk) {
  const uint64_t t0 = phase_now(ctx);
  struct Done {
    cmtv_ctx* c;
    uint64_t t;
    ~Done() { phase_add(c, kPhEarly, t); }
  } done{ctx, t0};
  clear_early_locked(ctx);  // whatever returns below stages nothing
  if (n == 0 || n > ctx->zc_max || ctx->live.size() != 1 || !ctx->early_sigs) return CMTV_OK;
  // the generic row kernels read their staging from mapped memory instead
  // (a copy's latency is most of their call); the quad-family forms gain the
  // HBM reads (10k: kernel 0.255 ms zero-copy, 0.220 ms from HBM)
  if (pk && (ed_form(ctx, n) == kFormRow4 || ed_form(ctx, n) == kFormRow)) return CMTV_OK;
  // nor is the copy worth its own latency for the keyed row kernel's
  // commits (150 validators: p50 0.0566 with it, 0.0534 without)
  if (!pk && keyed_form(ctx, n) == kKeyedRow) return CMTV_OK;
  // nor beside a pipeline call (bulk_now): the copy would queue behind its DMAs
  if (!pk && ((ctx->bulk_now && ctx->load_zc) || ctx->keyed_zc)) return CMTV_OK;
  CmtvDev& D = ctx->devs[ctx->live[0]];
  if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
  hipError_t e;
  // the previous polled launch may still read h_in's neighbour h_zin only,
  // but settle it anyway so the buffers below are never in use
  if ((e = settle_polled(D)) != hipSuccess) return hip_fail(e);
  // room for any layout of n signatures that can follow (keys, offsets,
  // templates, sign-bytes), so enqueue_shard never reallocates under the copy
  const size_t in_cap = 136 * n + 64 * 1024, dev_cap = in_cap + 400 * n;
  if ((e = D.h_in.ensure(in_cap)) != hipSuccess) return hip_fail(e);
  if ((e = D.d_in.ensure(dev_cap)) != hipSuccess) return hip_fail(e);
  // the keys where enqueue_shard's layout puts them for m = n signatures
  const size_t o_key = align_up(64 * n, 256);
  auto* hin = static_cast<uint8_t*>(D.h_in.p);
  auto* din = static_cast<uint8_t*>(D.d_in.p);
  // arrays in the caller's cmtv_alloc_pinned memory go to the device by DMA
  // straight from there (no host copy: 640 KB of signatures at 10k); the
  // others through h_in as before
  const bool sig_pinned = pinned_holds_locked(ctx, sigs, 64 * n);
  const bool pk_pinned = pk && pinned_holds_locked(ctx, pk, 32 * n);
  if (!sig_pinned) std::memcpy(hin, sigs, 64 * n);
  if (pk && !pk_pinned) std::memcpy(hin + o_key, pk, 32 * n);
  if (!sig_pinned && pk && !pk_pinned) {  // one copy of both
    e = hipMemcpyAsync(din, hin, o_key + 32 * n, hipMemcpyHostToDevice, D.stream);
  } else {
    e = hipMemcpyAsync(din, sig_pinned ? sigs : hin, 64 * n, hipMemcpyHostToDevice, D.stream);
    if (e == hipSuccess && pk)
      e = hipMemcpyAsync(din + o_key, pk_pinned ? pk : hin + o_key, 32 * n, hipMemcpyHostToDevice, D.stream);
  }
  if (e != hipSuccess) return hip_fail(e);
  D.early_src = sigs;
  D.early_pk = pk;
  D.early_n = n;
  return CMTV_OK;
}

// The single-device _device entry points run on devs[0] (their inputs are
// its memory): once it is retired they return CMTV_ENODEV rather than launch
// on a device that returned a HIP error. (Key generation and signing take
// host buffers and run on the first live device.)
static int dev0_usable(const cmtv_ctx* ctx) { return ctx->devs[0].failed ? CMTV_ENODEV : CMTV_OK; }

// A single-device _device call's result: CMTV_FAULT_AT's failure belongs to
// this call only, so the flag that marks it is cleared here (run_host_batch
// and sharded_device clear it on their own paths).
static int single_device_rc(cmtv_ctx* ctx, int rc) {
  ctx->fault_pending = false;
  return rc;
}

// Early-staged signatures (stage_sigs_early_locked) are valid only inside the
// lock hold of the cmtv_verify_commit call that staged them: every new hold
// forgets them, so a later call can never take stale device bytes for its own
// (the caller may refill the same buffer, and d_in / h_in may have been
// rewritten by another entry point meanwhile).
void clear_early_locked(cmtv_ctx* ctx) {
  for (auto& D : ctx->devs) {
    D.early_src = D.early_pk = nullptr;
    D.early_n = 0;
  }
}

int ctx_lock(cmtv_ctx* ctx, std::unique_lock<std::mutex>& lk) {
  ctx->lock_waiters.fetch_add(1, std::memory_order_relaxed);
  lk = std::unique_lock<std::mutex>(ctx->mu);
  ctx->lock_waiters.fetch_sub(1, std::memory_order_relaxed);
  clear_early_locked(ctx);
  // the forms of this hold's launches see one answer (keyed_form, ed_form)
  ctx->bulk_now = ctx->bulk_busy.load(std::memory_order_relaxed) > 0;
  ctx->under_load = ctx->bulk_now && ctx->lat_window_ns && ctx->load_form;
  return hipSetDevice(ctx->devs[0].ordinal) == hipSuccess ? CMTV_OK : CMTV_ENODEV;
}

void bulk_relock(cmtv_ctx* ctx, std::unique_lock<std::mutex>& lk) {
  // std::mutex is not fair: a pipeline thread that re-locks right after each
  // release can hold a 150-validator call off for several of its chunk
  // submissions (round 6: the under-load call's p99 was its wait before the
  // launch). Waiters go first, for at most 200 us.
  if (ctx->lock_waiters.load(std::memory_order_relaxed) > 0) {
    const auto t0 = std::chrono::steady_clock::now();
    while (ctx->lock_waiters.load(std::memory_order_relaxed) > 0 &&
           std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200))
      std::this_thread::yield();
  }
  lk.lock();
}

uint32_t ctx_default_mode(const cmtv_ctx* ctx) { return ctx->default_mode; }

// ---------------------------------------------------------------- lifecycle

static int init_device(cmtv_ctx* ctx, CmtvDev& D) {
  if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
  hipError_t e = hipStreamCreateWithFlags(&D.stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&D.scratch.done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&D.done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipMalloc(&D.d_diag, kDiagWords * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemsetAsync(D.d_diag, 0, kDiagWords * sizeof(uint32_t), D.stream);
  if (e == hipSuccess) e = hipMalloc(&D.d_rowslots, (size_t)kRowSlots * kRowSlotWords * sizeof(uint32_t));
  if (e == hipSuccess)
    e = hipMemsetAsync(D.d_rowslots, 0, (size_t)kRowSlots * kRowSlotWords * sizeof(uint32_t), D.stream);
  if (e == hipSuccess) e = hipMalloc(&D.d_btab, kBtabWords * sizeof(uint32_t));
  if (e == hipSuccess) e = launch_btab_init(D.d_btab, D.stream);
  uint32_t prog[SR_PREFIX_WORDS];
  ctx->sr_nops = sr_prefix_state(prog);
  if (ctx->sr_nops <= 0 && e == hipSuccess) e = hipErrorInvalidValue;
  if (e == hipSuccess) e = hipMalloc(&D.d_srprog, sizeof(prog));
  if (e == hipSuccess) e = hipMemcpyAsync(D.d_srprog, prog, sizeof(prog), hipMemcpyHostToDevice, D.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(D.stream);
  return e == hipSuccess ? CMTV_OK : hip_fail(e);
}

static void bulk_lane_release(CmtvDev& D);

static void release_device(CmtvDev& D) {
  (void)hipSetDevice(D.ordinal);
  if (D.stream) (void)hipStreamSynchronize(D.stream);
  bulk_lane_release(D);
  D.scratch.buf.release();
  D.d_in.release();
  D.d_out.release();
  D.d_all.release();
  D.h_in.release();
  D.h_out.release();
  D.h_zc.release();
  D.h_tags.release();
  D.d_tags = nullptr;
  D.h_zin.release();
  if (D.d_btab) (void)hipFree(D.d_btab);
  if (D.d_srprog) (void)hipFree(D.d_srprog);
  if (D.d_diag) (void)hipFree(D.d_diag);
  D.d_diag = nullptr;
  if (D.d_rowslots) (void)hipFree(D.d_rowslots);
  D.d_rowslots = nullptr;
  D.d_btab = nullptr;
  D.d_srprog = nullptr;
  D.timing.release();
  for (uint32_t k = 0; k < kRowSlots; k++) {
    if (D.row_ev[k]) (void)hipEventDestroy(D.row_ev[k]);
    D.row_ev[k] = nullptr;
    D.row_pending[k] = false;
  }
  if (D.scratch.done) (void)hipEventDestroy(D.scratch.done);
  if (D.done) (void)hipEventDestroy(D.done);
  if (D.poll_ev) (void)hipEventDestroy(D.poll_ev);
  D.poll_ev = nullptr;
  D.poll_pending = false;
  if (D.stream) (void)hipStreamDestroy(D.stream);
  D.scratch.done = D.done = nullptr;
  D.scratch.used = false;
  D.stream = nullptr;
}

// CMTV_FORM: comma-separated form names, a debug knob for tests and A/B runs
// (every other size keeps its band): row4 | row | oct2 | quad | lane (Ed25519;
// quad and lane also sr25519) and krow | kquad | klane (registered keys). An
// unknown name is reported once on stderr and ignored.
static void parse_forms(cmtv_ctx* ctx, const char* v) {
  static const struct {
    const char* name;
    bool keyed;
    uint32_t form;
  } kNames[] = {{"row4", false, kFormRow4}, {"row", false, kFormRow},   {"oct2", false, kFormOct2},
                {"quad", false, kFormQuad}, {"lane", false, kFormLane}, {"krow", true, kKeyedRow},
                {"kquad", true, kKeyedQuad}, {"klane", true, kKeyedLane}};
  std::string list(v);
  size_t p = 0;
  while (p <= list.size()) {
    size_t q = list.find(',', p);
    if (q == std::string::npos) q = list.size();
    const std::string tok = list.substr(p, q - p);
    p = q + 1;
    if (tok.empty()) continue;
    bool known = false;
    for (const auto& k : kNames)
      if (tok == k.name) {
        (k.keyed ? ctx->force_keyed : ctx->force_form) = k.form;
        known = true;
      }
    if (!known) std::fprintf(stderr, "cmtverify: CMTV_FORM: unknown form '%s' ignored\n", tok.c_str());
  }
}

static void read_env(cmtv_ctx* ctx) {
  if (const char* f = std::getenv("CMTV_FORM")) parse_forms(ctx, f);
  if (const char* hp = std::getenv("CMTV_HS_PRE")) {
    // 0..16 comb positions; anything else keeps the kernel's default
    char* end = nullptr;
    const long v = std::strtol(hp, &end, 10);
    if (end != hp && *end == 0 && v >= 0 && v <= 16) ctx->hs_tune = (uint32_t)(v + 1);
  }
  if (const char* lc = std::getenv("CMTV_LANE_CHUNK")) {
    const size_t v = (size_t)std::strtoull(lc, nullptr, 10) / 64 * 64;
    if (v >= 64 && v <= kChunk) ctx->lane_chunk = v;
  }
  if (const char* sm = std::getenv("CMTV_SHARD_MIN")) ctx->shard_min = (size_t)std::strtoull(sm, nullptr, 10);
  if (const char* fa = std::getenv("CMTV_FAULT_AT")) ctx->fault_at = (uint64_t)std::strtoull(fa, nullptr, 10);
  if (const char* fw = std::getenv("CMTV_FORCE_WIDE")) ctx->force_wide = fw[0] == '1';
  if (const char* nf = std::getenv("CMTV_NO_SB_FUSE")) ctx->sb_fuse = nf[0] != '1';
  if (const char* nz = std::getenv("CMTV_NO_ZC_IN")) ctx->zc_in = nz[0] != '1';
  if (const char* zh = std::getenv("CMTV_ZC_HOST_IN")) ctx->zc_host_in = zh[0] != '0';
  if (const char* es = std::getenv("CMTV_EARLY_SIGS")) ctx->early_sigs = es[0] != '0';
  if (const char* hp = std::getenv("CMTV_HOST_POLL")) ctx->host_poll = std::atoi(hp) != 0;
  if (const char* kl = std::getenv("CMTV_FORCE_K_LATE")) ctx->keyed_wait = kl[0] == '1' ? 0u : kKeyedWaitDefault;
  if (const char* mw = std::getenv("CMTV_KEYED_BATCH_MIN_WAVES")) {
    const long v = std::strtol(mw, nullptr, 10);
    if (v >= 1 && v <= (1l << 20)) ctx->keyed_batch_min_waves = (uint32_t)v;
  }
  if (const char* rf = std::getenv("CMTV_ROW_FENCE")) ctx->row_fence = rf[0] != '0';
  if (const char* hp = std::getenv("CMTV_HOST_PHASES")) ctx->phases_on = hp[0] == '1';
  if (const char* tm = std::getenv("CMTV_TIMING")) {
    const long v = std::strtol(tm, nullptr, 10);
    ctx->timing_every = v < 0 ? 0u : (uint32_t)std::min<long>(v, 1l << 20);
  }
  if (const char* fs = std::getenv("CMTV_FAULT_SYNC_DEV")) {
    char* end = nullptr;
    const long g = std::strtol(fs, &end, 10);
    if (end != fs && g >= 0) ctx->fault_sync_dev = g;
  }
  ctx->force_rccl = std::getenv("CMTV_FORCE_RCCL") != nullptr;
  if (const char* rl = std::getenv("CMTV_RCCL_LIB")) ctx->rccl_lib = rl;
  ctx->no_rccl = std::getenv("CMTV_NO_RCCL") != nullptr;
  ctx->no_rccl_fallback = std::getenv("CMTV_NO_RCCL_FALLBACK") != nullptr;
  if (const char* v = std::getenv("CMTV_HOST_THREADS")) {
    const long t = std::strtol(v, nullptr, 10);
    if (t >= 1 && t <= 256) ctx->host_threads = (unsigned)t;
  }
  if (const char* v = std::getenv("CMTV_PIPE_MIN")) ctx->pipe_min = (size_t)std::strtoull(v, nullptr, 10);
  if (const char* v = std::getenv("CMTV_PIPE_CHUNK")) {
    const size_t c = (size_t)std::strtoull(v, nullptr, 10);
    if (c >= 64 && c <= (1u << 24)) ctx->pipe_chunk = c;
  }
  if (const char* v = std::getenv("CMTV_PIPE_SLOTS")) {
    const long k = std::strtol(v, nullptr, 10);
    if (k >= 2 && k <= kBulkSlotsMax) ctx->pipe_slots = (int)k;
  }
  if (const char* v = std::getenv("CMTV_PIPELINE")) ctx->pipe_on = v[0] != '0';
  if (const char* v = std::getenv("CMTV_PIPE_DIRECT")) ctx->pipe_direct = v[0] != '0';
  if (const char* v = std::getenv("CMTV_SPEC_MIN")) {
    const long x = std::strtol(v, nullptr, 10);
    if (x > 0) ctx->spec_min = (uint32_t)x;
  }
  if (const char* v = std::getenv("CMTV_SPEC")) {
    if (v[0] == '0') ctx->spec_min = 0;
  }
  if (const char* v = std::getenv("CMTV_LAT_WINDOW_MS")) ctx->lat_window_ns = 1'000'000ull * std::strtoull(v, nullptr, 10);
  if (const char* v = std::getenv("CMTV_LOAD_FORM")) ctx->load_form = v[0] != '0';
  if (const char* v = std::getenv("CMTV_LOAD_ZC")) ctx->load_zc = v[0] != '0';
  if (const char* v = std::getenv("CMTV_LOAD_POLL")) ctx->load_nopoll = v[0] == '0';
  if (const char* v = std::getenv("CMTV_QUAD_POLL")) ctx->quad_poll = v[0] == '1';
  if (const char* v = std::getenv("CMTV_KEYED_ZC")) ctx->keyed_zc = v[0] != '0';
  if (const char* v = std::getenv("CMTV_SPIN_WAIT")) ctx->spin_wait = v[0] == '1';
  if (const char* v = std::getenv("CMTV_PREP_STREAM")) ctx->prep_stream = v[0] != '0';
  if (const char* v = std::getenv("CMTV_ONE_EXEC")) ctx->one_exec = v[0] == '1';
  if (const char* v = std::getenv("CMTV_BULK_BM_DIRECT")) ctx->bulk_bm_direct = v[0] == '1';
  if (const char* v = std::getenv("CMTV_SPLIT_SUBMIT")) ctx->split_submit = v[0] != '0';
  if (const char* v = std::getenv("CMTV_CALL_TRACE")) {
    ctx->call_trace = v[0] == '1' || v[0] == '2';
    ctx->call_trace_loaded_only = v[0] == '2';  // only calls beside a pipeline call
  }
  if (const char* v = std::getenv("CMTV_LAT_ISOLATE")) ctx->lat_isolate = v[0] != '0';
  if (const char* v = std::getenv("CMTV_LAT_RESERVE_CUS")) {
    const long k = std::strtol(v, nullptr, 10);
    if (k >= 1 && k <= 64) ctx->lat_reserve_cus = (uint32_t)k;
  }
  if (const char* dm = std::getenv("CMTV_RCCL_DRAIN_MS")) {
    const long v = std::strtol(dm, nullptr, 10);
    if (v >= 1 && v <= 600000) ctx->rccl_drain_ms = (uint32_t)v;
  }
}

// The bitmap communicator over the live devices (rank = position in
// ctx->live), when their ordinals are distinct and librccl loads; a one-rank
// communicator only under CMTV_FORCE_RCCL (the RCCL path on a one-GPU box).
// Otherwise gathers use peer copies. Called at open and after a device is
// retired (the old communicator included it).
static void rebuild_comm(cmtv_ctx* ctx) {
  const Rccl& R = rccl(ctx->rccl_lib);
  drop_comms(ctx, false);
  ctx->rccl = false;
  std::vector<int> ords;
  for (size_t d : ctx->live) ords.push_back(ctx->devs[d].ordinal);
  std::vector<int> sorted = ords;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  // a repeated ordinal gets a communicator only from a library named by
  // CMTV_RCCL_LIB under CMTV_FORCE_RCCL (the one-GPU rehearsal of the
  // multi-rank path); the system RCCL refuses duplicate devices
  const bool repeat_ok = ctx->force_rccl && !ctx->rccl_lib.empty();
  const bool want = !ctx->rccl_broken && (ords.size() > 1 ? ((distinct || repeat_ok) && !ctx->no_rccl)
                                                           : (ords.size() == 1 && ctx->force_rccl));
  if (want && R.ok) {
    std::vector<ncclComm_t> comms(ords.size(), nullptr);
    if (R.CommInitAll(comms.data(), (int)ords.size(), ords.data()) == 0) {
      for (size_t g = 0; g < ords.size(); g++) ctx->devs[ctx->live[g]].comm = comms[g];
      ctx->rccl = true;
    }
  }
  ctx->stats.rccl = ctx->rccl ? 1 : 0;
  (void)hipSetDevice(ctx->devs[ctx->live.empty() ? 0 : ctx->live[0]].ordinal);
}

// CMTVERIFY_DEVICES: "0,1,2" or "all" (or unset: every visible device)
static std::vector<int> env_devices(int ndev) {
  std::vector<int> out;
  const char* v = std::getenv("CMTVERIFY_DEVICES");
  if (v && *v && std::strcmp(v, "all") != 0) {
    const char* p = v;
    while (*p) {
      char* end = nullptr;
      const long x = std::strtol(p, &end, 10);
      if (end == p) return {};
      out.push_back((int)x);
      p = end;
      while (*p == ',' || *p == ' ') p++;
    }
    return out;
  }
  for (int i = 0; i < ndev; i++) out.push_back(i);
  return out;
}

static int open_ctx(const cmtv_config* cfg, const std::vector<int>& ords, cmtv_ctx** out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return CMTV_ENODEV;
  if (ords.empty() || ords.size() > (size_t)kMaxDevices) return CMTV_EINVAL;
  uint32_t cus = UINT32_MAX;
  for (int o : ords) {
    if (o < 0 || o >= ndev) return CMTV_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, o) != hipSuccess) return CMTV_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CMTV_ENODEV;
    cus = std::min(cus, (uint32_t)std::max(prop.multiProcessorCount, 1));
  }
  auto* ctx = new (std::nothrow) cmtv_ctx();
  if (!ctx) return CMTV_ENOMEM;
  ctx->cus = cus;
  ctx->default_mode = cfg ? cfg->default_mode : CMTV_MODE_GO_STDLIB;
  if (!cfg) {
    const char* m = std::getenv("CMTVERIFY_MODE");
    if (m && std::strcmp(m, "zip215") == 0) ctx->default_mode = CMTV_MODE_ZIP215;
  }
  read_env(ctx);
  ctx->devs.resize(ords.size());
  for (size_t g = 0; g < ords.size(); g++) ctx->devs[g].ordinal = ords[g];
  for (auto& D : ctx->devs) {
    const int rc = init_device(ctx, D);
    if (rc != CMTV_OK) {
      cmtv_close(ctx);
      return rc;
    }
  }
  ctx->stats.n_devices = (uint32_t)ords.size();
  for (size_t g = 0; g < ords.size(); g++) ctx->live.push_back(g);
  // CMTV_FAULT_DEV=g: the g-th device's launches fail (re-shard test knob)
  if (const char* fd = std::getenv("CMTV_FAULT_DEV")) {
    char* end = nullptr;
    const long g = std::strtol(fd, &end, 10);
    if (end != fd && g >= 0 && (size_t)g < ords.size()) ctx->devs[(size_t)g].inject_fault = true;
  }
  if (ords.size() > 1) {
    for (size_t g = 0; g < ords.size(); g++) {  // peer access for the copy gathers
      (void)hipSetDevice(ords[g]);
      for (size_t h = 0; h < ords.size(); h++)
        if (ords[h] != ords[g]) (void)hipDeviceEnablePeerAccess(ords[h], 0);
    }
    (void)hipGetLastError();  // "already enabled" is not an error here
  }
  rebuild_comm(ctx);
  (void)hipSetDevice(ords[0]);
  *out = ctx;
  return CMTV_OK;
}

}  // namespace cmtv

using namespace cmtv;

extern "C" {

int cmtv_abi_version(void) { return CMTV_ABI_VERSION; }

const char* cmtv_strerror(int code) {
  switch (code) {
    case CMTV_OK: return "ok";
    case CMTV_EINVAL: return "invalid argument";
    case CMTV_ENODEV: return "no usable gfx950 device";
    case CMTV_ENOMEM: return "out of device or pinned host memory";
    case CMTV_EHIP: return "HIP runtime error";
    case CMTV_ERCCL: return "collective communication error";
    case CMTV_ECOMMIT: return "commit verification failed";
    default: return "unknown error";
  }
}

int cmtv_open(const cmtv_config* cfg, cmtv_ctx** out) {
  if (!out) return CMTV_EINVAL;
  *out = nullptr;
  if (cfg && (cfg->flags != 0 || cfg->default_mode > CMTV_MODE_ZIP215)) return CMTV_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return CMTV_ENODEV;
  int dev = 0;
  if (cfg && cfg->device >= 0) {
    dev = cfg->device;
  } else if (hipGetDevice(&dev) != hipSuccess) {
    dev = 0;
  }
  return open_ctx(cfg, {dev}, out);
}

int cmtv_open_devices(const cmtv_config* cfg, const int32_t* devices, size_t n_devices, cmtv_ctx** out) {
  if (!out) return CMTV_EINVAL;
  *out = nullptr;
  if (cfg && (cfg->flags != 0 || cfg->default_mode > CMTV_MODE_ZIP215)) return CMTV_EINVAL;
  if (n_devices > (size_t)kMaxDevices || (n_devices && !devices)) return CMTV_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return CMTV_ENODEV;
  std::vector<int> ords = n_devices ? std::vector<int>(devices, devices + n_devices) : env_devices(ndev);
  if (ords.empty()) return CMTV_EINVAL;
  return open_ctx(cfg, ords, out);
}

void cmtv_close(cmtv_ctx* ctx) {
  if (!ctx) return;
  if (ctx->phases_on) {
    static const char* names[kPhCount] = {"prepare",   "stage",     "launch",      "wait",      "post",       "replay",
                                          "pipe_plan", "pipe_pack", "pipe_submit", "pipe_wait", "pipe_replay",
                                          "keyset",    "early",     "pipe_cut"};
    std::fprintf(stderr, "{\"cmtv_host_phases_us\": {");
    for (int p = 0; p < kPhCount; p++)
      std::fprintf(stderr, "%s\"%s\": %.3f", p ? ", " : "", names[p],
                   ctx->phase_calls ? 1e-3 * (double)ctx->phase_ns[p] / (double)ctx->phase_calls : 0.0);
    std::fprintf(stderr, "}, \"calls\": %llu}\n", (unsigned long long)ctx->phase_calls);
  }
  if (ctx->call_trace && !ctx->trace_rows.empty()) {
    static const char* seg[5] = {"to_lock", "to_launch", "gpu_and_wake", "post", "device_events"};
    std::fprintf(stderr, "{\"cmtv_call_trace_us\": {\"calls\": %zu", ctx->trace_rows.size());
    for (int k = 0; k < 5; k++) {
      std::vector<uint64_t> v;
      for (auto& r : ctx->trace_rows) v.push_back(r[k]);
      std::sort(v.begin(), v.end());
      auto q = [&](double f) { return 1e-3 * (double)v[std::min(v.size() - 1, (size_t)(f * (double)v.size()))]; };
      std::fprintf(stderr, ", \"%s\": [%.1f, %.1f, %.1f, %.1f]", seg[k], q(0.5), q(0.9), q(0.99), q(1.0));
    }
    // the slowest tenth of calls: which segment took their excess
    std::vector<size_t> idx(ctx->trace_rows.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
    auto total = [&](size_t i) { auto& r = ctx->trace_rows[i]; return r[0] + r[1] + r[2] + r[3]; };
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return total(a) < total(b); });
    std::fprintf(stderr, ", \"slowest_1pct\": [");
    const size_t from = idx.size() - std::max<size_t>(1, idx.size() / 100);
    for (size_t j = from; j < idx.size(); j++) {
      auto& r = ctx->trace_rows[idx[j]];
      std::fprintf(stderr, "%s[%.1f, %.1f, %.1f, %.1f, %.1f]", j > from ? ", " : "", 1e-3 * r[0], 1e-3 * r[1],
                   1e-3 * r[2], 1e-3 * r[3], 1e-3 * r[4]);
    }
    std::fprintf(stderr, "]}}\n");
  }
  for (auto& ev : ctx->trace_ev)
    if (ev) (void)hipEventDestroy(ev);
  ctx->pool.reset();
  for (auto& b : ctx->pinned) (void)hipHostFree(reinterpret_cast<void*>(b.first));  // the caller's leftovers
  ctx->pinned.clear();
  pipe_workspace_free(ctx->pipe_ws);
  ctx->pipe_ws = nullptr;
  for (auto& e : ctx->keysets) cmtv_keyset_free(e.second);
  ctx->keysets.clear();
  for (auto* z : ctx->zombies) cmtv_keyset_free(z);
  ctx->zombies.clear();
  drop_comms(ctx, false);
  for (auto& D : ctx->devs) release_device(D);
  delete ctx;
}

void* cmtv_stream(cmtv_ctx* ctx) { return ctx ? static_cast<void*>(ctx->devs[0].stream) : nullptr; }

int cmtv_device_count(const cmtv_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int cmtv_device_ordinal(const cmtv_ctx* ctx, int g) {
  if (!ctx || g < 0 || g >= (int)ctx->devs.size()) return CMTV_EINVAL;
  return ctx->devs[g].ordinal;
}

void* cmtv_device_stream(cmtv_ctx* ctx, int g) {
  if (!ctx || g < 0 || g >= (int)ctx->devs.size()) return nullptr;
  return static_cast<void*>(ctx->devs[g].stream);
}

int cmtv_sync(cmtv_ctx* ctx) {
  if (!ctx) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  for (auto& D : ctx->devs) {
    if (D.failed) continue;
    if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
    const hipError_t e = hipStreamSynchronize(D.stream);
    if (e != hipSuccess) return hip_fail(e);
  }
  harvest(ctx, false);
  (void)hipSetDevice(ctx->devs[0].ordinal);
  return CMTV_OK;
}

// the kernels' diagnostic counters of every usable device, summed
static void read_diag(cmtv_ctx* ctx) {
  uint64_t late = 0;
  for (auto& D : ctx->devs) {
    if (D.failed || !D.d_diag) continue;
    (void)hipSetDevice(D.ordinal);
    uint32_t w[kDiagWords] = {};
    if (hipMemcpy(w, D.d_diag, sizeof(w), hipMemcpyDeviceToHost) == hipSuccess) late += w[kDiagLateK];
  }
  ctx->stats.late_k_waves = late;
}

int cmtv_stats_get(cmtv_ctx* ctx, cmtv_stats* out) {
  if (!ctx || !out) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  harvest(ctx, true);
  read_diag(ctx);
  (void)hipSetDevice(ctx->devs[0].ordinal);
  ctx->stats.cache_entries = ctx->cache.size();
  ctx->stats.live_devices = (uint32_t)ctx->live.size();
  *out = ctx->stats;
  return CMTV_OK;
}

int cmtv_device_stats_get(cmtv_ctx* ctx, int g, cmtv_device_stats* out) {
  if (!ctx || !out || g < 0 || g >= (int)ctx->devs.size()) return CMTV_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  harvest(ctx, true);
  CmtvDev& D = ctx->devs[(size_t)g];
  std::memset(out, 0, sizeof(*out));
  out->ordinal = D.ordinal;
  out->failed = D.failed ? 1 : 0;
  out->calls = D.calls;
  out->signatures = D.signatures;
  out->kernel_launches = D.launches;
  out->device_ms = D.device_ms;
  out->timed_calls = D.timed_calls;
  (void)hipSetDevice(ctx->devs[0].ordinal);
  return CMTV_OK;
}

int cmtv_verdict_cache(cmtv_ctx* ctx, size_t max_entries) {
  if (!ctx || max_entries > (1u << 26)) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->cache.reset(max_entries);
  return CMTV_OK;
}

int cmtv_verify_ed25519(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                        const uint32_t* msg_off, uint32_t mode, uint8_t* out_valid, uint64_t* out_bitmap) {
  if (!ctx || mode > CMTV_MODE_ZIP215 || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!pk || !sig || !msg_off || (!msg && msg_off[n] != 0) || (!out_valid && !out_bitmap)) return CMTV_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (msg_off[i + 1] < msg_off[i]) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  return verify_host_locked(ctx, n, pk, sig, msg, msg_off, mode, out_valid, out_bitmap);
}

int cmtv_verify_ed25519_device(cmtv_ctx* ctx, size_t n, const void* d_pk, const void* d_sig, const void* d_msg,
                               const void* d_msg_off, uint32_t mode, void* d_valid, void* d_bitmap, void* stream) {
  if (!ctx || mode > CMTV_MODE_ZIP215 || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!d_pk || !d_sig || !d_msg || !d_msg_off || (!d_valid && !d_bitmap)) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  if (dev0_usable(ctx) != CMTV_OK) return CMTV_ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
  return single_device_rc(
      ctx, enqueue_verify(ctx, ctx->devs[0], n, static_cast<const uint8_t*>(d_pk), static_cast<const uint8_t*>(d_sig),
                          static_cast<const uint8_t*>(d_msg), static_cast<const uint32_t*>(d_msg_off), mode,
                          static_cast<uint8_t*>(d_valid), static_cast<uint64_t*>(d_bitmap), s));
}

int cmtv_verify_sr25519(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                        const uint32_t* msg_off, uint8_t* out_valid, uint64_t* out_bitmap) {
  if (!ctx || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!pk || !sig || !msg_off || (!msg && msg_off[n] != 0) || (!out_valid && !out_bitmap)) return CMTV_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (msg_off[i + 1] < msg_off[i]) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  return verify_host_locked(ctx, n, pk, sig, msg, msg_off, kModeSr25519, out_valid, out_bitmap);
}

int cmtv_verify_sr25519_device(cmtv_ctx* ctx, size_t n, const void* d_pk, const void* d_sig, const void* d_msg,
                               const void* d_msg_off, void* d_valid, void* d_bitmap, void* stream) {
  if (!ctx || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!d_pk || !d_sig || !d_msg || !d_msg_off || (!d_valid && !d_bitmap)) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  if (dev0_usable(ctx) != CMTV_OK) return CMTV_ENODEV;
  return single_device_rc(
      ctx, enqueue_verify(ctx, ctx->devs[0], n, static_cast<const uint8_t*>(d_pk), static_cast<const uint8_t*>(d_sig),
                          static_cast<const uint8_t*>(d_msg), static_cast<const uint32_t*>(d_msg_off), kModeSr25519,
                          static_cast<uint8_t*>(d_valid), static_cast<uint64_t*>(d_bitmap),
                          static_cast<hipStream_t>(stream)));
}

}  // extern "C"

namespace cmtv {

// Shared by the two sharded device-resident entry points: shard g's inputs on
// device g, each verified on its device's stream, then the bitmap gather.
static int sharded_device(cmtv_ctx* ctx, const cmtv_keyset* ks, const size_t* n_shard, const void* const* d_keys,
                          const void* const* d_sig, const void* const* d_msg, const void* const* d_off,
                          uint32_t mode, void* const* d_valid, void* const* d_bitmap_all, size_t* words_per_shard,
                          bool gather = true) {
  const size_t G = ctx->devs.size();
  // the caller's inputs live on every device: a retired one cannot take part
  if (ctx->live.size() != G) return CMTV_ENODEV;
  size_t W = 0;
  for (size_t g = 0; g < G; g++) {
    if (n_shard[g] > (1ull << 31)) return CMTV_EINVAL;
    if (n_shard[g] && (!d_keys[g] || !d_sig[g] || !d_msg[g] || !d_off[g])) return CMTV_EINVAL;
    if (!d_bitmap_all[g]) return CMTV_EINVAL;
    W = std::max(W, (n_shard[g] + 63) / 64);
  }
  if (words_per_shard) *words_per_shard = W;
  if (W == 0) return CMTV_OK;
  uint64_t* bufs[kMaxDevices];
  hipError_t e;
  for (size_t g = 0; g < G; g++) {
    CmtvDev& D = ctx->devs[g];
    if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
    bufs[g] = static_cast<uint64_t*>(d_bitmap_all[g]);
    // independent batches (no gather): device g's bitmap is its own words
    uint64_t* own_bm = gather ? bufs[g] + g * W : bufs[g];
    // words of this shard beyond its signatures stay zero (quad kernels write
    // whole 16-bit slices, lane kernels whole words; a short shard leaves the
    // rest of its W words untouched)
    const size_t own = (n_shard[g] + 63) / 64;
    if (gather && own < W && (e = hipMemsetAsync(own_bm + own, 0, 8 * (W - own), D.stream)) != hipSuccess)
      return hip_fail(e);
    uint8_t* dv = d_valid ? static_cast<uint8_t*>(d_valid[g]) : nullptr;
    int rc;
    if (ks)
      rc = enqueue_verify_keyed(ctx, D, ks->dev[g], ks->n, n_shard[g], static_cast<const uint32_t*>(d_keys[g]),
                                static_cast<const uint8_t*>(d_sig[g]), static_cast<const uint8_t*>(d_msg[g]),
                                static_cast<const uint32_t*>(d_off[g]), mode, dv, own_bm, D.stream);
    else
      rc = enqueue_verify(ctx, D, n_shard[g], static_cast<const uint8_t*>(d_keys[g]),
                          static_cast<const uint8_t*>(d_sig[g]), static_cast<const uint8_t*>(d_msg[g]),
                          static_cast<const uint32_t*>(d_off[g]), mode, dv, own_bm, D.stream);
    if (rc != CMTV_OK) {
      // a device's own HIP error takes it out of the rotation (host batches
      // re-plan over the others); this call fails: its inputs were there
      const bool injected = ctx->fault_pending;
      ctx->fault_pending = false;
      if (rc == CMTV_EHIP && !injected && G > 1) retire_device(ctx, g);
      (void)hipSetDevice(ctx->devs[0].ordinal);
      return rc;
    }
  }
  if (!gather) {
    (void)hipSetDevice(ctx->devs[0].ordinal);
    return CMTV_OK;
  }
  if (G > 1) ctx->stats.sharded_calls++;
  const int rc = gather_bitmaps(ctx, ctx->live.data(), G, W, bufs);
  (void)hipSetDevice(ctx->devs[0].ordinal);
  return rc;
}

}  // namespace cmtv

extern "C" {

int cmtv_verify_ed25519_sharded_device(cmtv_ctx* ctx, const size_t* n_shard, const void* const* d_pk,
                                       const void* const* d_sig, const void* const* d_msg,
                                       const void* const* d_msg_off, uint32_t mode, void* const* d_valid,
                                       void* const* d_bitmap_all, size_t* words_per_shard) {
  if (!ctx || mode > CMTV_MODE_ZIP215 || !n_shard || !d_pk || !d_sig || !d_msg || !d_msg_off || !d_bitmap_all)
    return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  return sharded_device(ctx, nullptr, n_shard, d_pk, d_sig, d_msg, d_msg_off, mode, d_valid, d_bitmap_all,
                        words_per_shard);
}

int cmtv_verify_ed25519_multi_device(cmtv_ctx* ctx, const size_t* n_dev, const void* const* d_pk,
                                     const void* const* d_sig, const void* const* d_msg,
                                     const void* const* d_msg_off, uint32_t mode, void* const* d_valid,
                                     void* const* d_bitmap) {
  if (!ctx || mode > CMTV_MODE_ZIP215 || !n_dev || !d_pk || !d_sig || !d_msg || !d_msg_off || !d_bitmap)
    return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  return sharded_device(ctx, nullptr, n_dev, d_pk, d_sig, d_msg, d_msg_off, mode, d_valid, d_bitmap, nullptr,
                        false);
}

int cmtv_verify_ed25519_indexed_sharded_device(cmtv_ctx* ctx, const cmtv_keyset* ks, const size_t* n_shard,
                                               const void* const* d_key_idx, const void* const* d_sig,
                                               const void* const* d_msg, const void* const* d_msg_off,
                                               uint32_t mode, void* const* d_valid, void* const* d_bitmap_all,
                                               size_t* words_per_shard) {
  if (!ctx || !ks || ks->ctx != ctx || mode > CMTV_MODE_ZIP215 || !n_shard || !d_key_idx || !d_sig || !d_msg ||
      !d_msg_off || !d_bitmap_all)
    return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  return sharded_device(ctx, ks, n_shard, d_key_idx, d_sig, d_msg, d_msg_off, mode, d_valid, d_bitmap_all,
                        words_per_shard);
}

int cmtv_register_keys_ex(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, uint32_t flags, cmtv_keyset** out) {
  if (!out) return CMTV_EINVAL;
  *out = nullptr;
  // 512 KiB of comb per key; 2^20 keys would already be 512 GiB (wide: 64 MiB
  // per key, 4096 keys = 256 GiB)
  if (!ctx || n_keys == 0 || n_keys > (1u << 20) || !pk || (flags & ~(uint32_t)CMTV_KEYS_WIDE)) return CMTV_EINVAL;
  if ((flags & CMTV_KEYS_WIDE) && n_keys > 4096) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  return cmtv::register_keys_locked(ctx, n_keys, pk, out, flags);
}

int cmtv_register_keys(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, cmtv_keyset** out) {
  return cmtv_register_keys_ex(ctx, n_keys, pk, 0, out);
}

int cmtv_keyset_cache(cmtv_ctx* ctx, size_t max_sets) {
  if (!ctx || max_sets > 4096) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  for (auto& D : ctx->devs) {
    (void)hipSetDevice(D.ordinal);
    (void)hipStreamSynchronize(D.stream);
  }
  while (ctx->keysets.size() > max_sets) {
    evict_keyset_locked(ctx, ctx->keysets.front().second);
    ctx->keysets.erase(ctx->keysets.begin());
  }
  ctx->keyset_cap = max_sets;
  (void)hipSetDevice(ctx->devs[0].ordinal);
  return CMTV_OK;
}

}  // extern "C"

namespace cmtv {

// keys per wide-comb build launch (prefix-product scratch = 20 MiB per key)
constexpr uint32_t kWideKeyChunk = 16;

// The wide combs of a key set on device D (current): 64 MiB per key.
static hipError_t build_wide(CmtvDev& D, cmtv_keyset::PerDev& K, size_t n_keys) {
  DevBuf scratch, bases;
  const size_t chunk = std::min<size_t>(n_keys, kWideKeyChunk);
  hipError_t e = hipMalloc(&K.d_wide, n_keys * kWideTableWords * sizeof(uint32_t));
  if (e == hipSuccess) e = scratch.ensure(chunk * kWideScratchWordsPerKey * sizeof(uint32_t));
  if (e == hipSuccess) e = bases.ensure(chunk * kWideBaseWordsPerKey * sizeof(uint32_t));
  for (size_t c = 0; e == hipSuccess && c < n_keys; c += kWideKeyChunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(kWideKeyChunk, n_keys - c);
    e = launch_wide_build(cn, K.d_pk + 8 * c, K.d_wide + c * kWideTableWords, static_cast<uint32_t*>(bases.p),
                          static_cast<uint32_t*>(scratch.p), D.stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(D.stream);
  scratch.release();
  bases.release();
  return e;
}

int register_keys_locked(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, cmtv_keyset** out, uint32_t flags) {
  auto* ks = new (std::nothrow) cmtv_keyset();
  if (!ks) return CMTV_ENOMEM;
  ks->ctx = ctx;
  ks->n = n_keys;
  ks->pk.assign(pk, pk + 32 * n_keys);
  ks->dev.resize(ctx->devs.size());
  for (size_t g = 0; g < ctx->devs.size(); g++) {
    CmtvDev& D = ctx->devs[g];
    auto& K = ks->dev[g];
    if (D.failed) continue;  // retired: never given work again
    (void)hipSetDevice(D.ordinal);
    DevBuf scratch;
    hipError_t e = hipMalloc(&K.d_pk, 32 * n_keys);
    if (e == hipSuccess) e = hipMalloc(&K.d_ok, n_keys);
    if (e == hipSuccess) e = hipMalloc(&K.d_tab, n_keys * (size_t)kCombWords * sizeof(uint32_t));
    if (e == hipSuccess)
      e = scratch.ensure((size_t)std::min<size_t>(n_keys, kCombKeyChunk) * kCombScratchWordsPerKey *
                         sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemcpyAsync(K.d_pk, pk, 32 * n_keys, hipMemcpyHostToDevice, D.stream);
    for (size_t c = 0; e == hipSuccess && c < n_keys; c += kCombKeyChunk) {
      const uint32_t cn = (uint32_t)std::min<size_t>(kCombKeyChunk, n_keys - c);
      e = launch_comb_build(cn, K.d_pk + 8 * c, K.d_ok + c, K.d_tab + c * (size_t)kCombWords,
                            static_cast<uint32_t*>(scratch.p), true, D.stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(D.stream);
    scratch.release();
    if (e == hipSuccess && (flags & CMTV_KEYS_WIDE)) e = build_wide(D, K, n_keys);
    if (e != hipSuccess) {
      cmtv_keyset_free(ks);
      (void)hipSetDevice(ctx->devs[0].ordinal);
      return hip_fail(e);
    }
  }
  (void)hipSetDevice(ctx->devs[0].ordinal);
  *out = ks;
  return CMTV_OK;
}

// A cached key set leaving the cache: freed now, or by the pipeline call
// that still has it pinned (keyset_unpin_locked).
static void evict_keyset_locked(cmtv_ctx* ctx, cmtv_keyset* ks) {
  if (ctx->guess_ks == ks) ctx->guess_ks = nullptr;
  if (ks->pins > 0) {
    ks->evicted = true;
    ctx->zombies.push_back(ks);
    return;
  }
  cmtv_keyset_free(ks);
}

void keyset_pin_locked(const cmtv_keyset* ks) { const_cast<cmtv_keyset*>(ks)->pins++; }

void keyset_unpin_locked(cmtv_ctx* ctx, const cmtv_keyset* cks) {
  auto* ks = const_cast<cmtv_keyset*>(cks);
  if (--ks->pins > 0 || !ks->evicted) return;
  ctx->zombies.erase(std::remove(ctx->zombies.begin(), ctx->zombies.end(), ks), ctx->zombies.end());
  cmtv_keyset_free(ks);
}

const cmtv_keyset* keyset_for_locked(cmtv_ctx* ctx, const uint8_t* pk32, size_t n_keys) {
  if (!ctx->keyset_cap || n_keys == 0) return nullptr;
  const size_t bytes = 32 * n_keys;
  auto remember = [&](const cmtv_keyset* k) {
    ctx->guess_pk = pk32;
    ctx->guess_n = n_keys;
    ctx->guess_ks = k;
    return k;
  };
  for (auto& e : ctx->keysets)  // compared in place: no copy of the keys per call
    if (e.first.size() == bytes && std::memcmp(e.first.data(), pk32, bytes) == 0) return remember(e.second);
  std::string key(reinterpret_cast<const char*>(pk32), bytes);
  cmtv_keyset* ks = nullptr;
  if (register_keys_locked(ctx, n_keys, pk32, &ks, 0) != CMTV_OK) return nullptr;  // generic path instead
  if (ctx->keysets.size() >= ctx->keyset_cap) {
    evict_keyset_locked(ctx, ctx->keysets.front().second);
    ctx->keysets.erase(ctx->keysets.begin());
  }
  ctx->keysets.emplace_back(std::move(key), ks);
  return remember(ks);
}

const cmtv_keyset* keyset_guess_locked(const cmtv_ctx* ctx, const uint8_t* pk32, size_t n_keys) {
  return ctx->guess_ks && ctx->guess_pk == pk32 && ctx->guess_n == n_keys ? ctx->guess_ks : nullptr;
}

uint32_t spec_min(const cmtv_ctx* ctx) { return ctx->spec_min; }

bool keyset_holds_locked(const cmtv_keyset* ks, const uint8_t* pk32, size_t n_keys) {
  return ks->n == n_keys && std::memcmp(ks->pk.data(), pk32, 32 * n_keys) == 0;
}

bool keyset_cache_enabled(const cmtv_ctx* ctx) { return ctx->keyset_cap != 0; }

// ---------------------------------------------------------------- bulk lanes

std::mutex& bulk_mutex(cmtv_ctx* ctx) { return ctx->bulk_mu; }

// CUs a masked bulk lane leaves to the latency stream (bulk_lane_init): a
// multiple of 8 (every XCD), at most a quarter of the device, 0 below 64 CUs
static uint32_t reserved_cus(const cmtv_ctx* ctx, uint32_t cus) {
  if (cus < 64) return 0;
  return std::min((ctx->lat_reserve_cus + 7) / 8 * 8, cus / 4 / 8 * 8);
}

static uint64_t now_ns_steady() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// CPUs this process may run on: the affinity mask, bounded by a cgroup v2
// CPU quota (cpu.max) when one is set
static unsigned usable_cpus() {
  unsigned n = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = (unsigned)CPU_COUNT(&set);
  if (n == 0) n = std::max(1u, std::thread::hardware_concurrency());
  std::ifstream f("/sys/fs/cgroup/cpu.max");
  std::string quota, period;
  if (f >> quota >> period && quota != "max") {
    const double q = std::atof(quota.c_str()), p = std::atof(period.c_str());
    if (q > 0 && p > 0) n = std::min(n, std::max(1u, (unsigned)(q / p)));
  }
  return n;
}

HostPool& host_pool(cmtv_ctx* ctx) {
  if (!ctx->pool) {
    // default: at most 16, and three CPUs short of a small CPU budget, so a
    // latency caller (consensus) and the HIP runtime's threads keep a CPU
    // under a cgroup quota (round 6, tools/gpu_r6aa.sh, 16-CPU quota, three
    // alternating rounds: latency_150_under_load p99 0.125-0.137 ms with 13
    // workers against 0.132-0.173 with 16)
    const unsigned u = usable_cpus();
    const unsigned t = ctx->host_threads ? ctx->host_threads : std::min(16u, u > 8 ? u - 3 : u);
    ctx->pool.reset(new HostPool(t));
  }
  return *ctx->pool;
}

PipeConfig pipe_config(const cmtv_ctx* ctx) {
  PipeConfig pc{ctx->pipe_min, ctx->pipe_chunk, ctx->pipe_slots, ctx->pipe_on, ctx->pipe_direct};
  pc.split_submit = ctx->split_submit;
  // a masked lane's round: the chunk scaled to the CUs it keeps (bulk_lane_init)
  const uint32_t reserved = reserved_cus(ctx, ctx->cus);
  pc.chunk_masked = ctx->cus > reserved
                        ? std::max<size_t>(64, ctx->pipe_chunk / ctx->cus * (ctx->cus - reserved))
                        : ctx->pipe_chunk;
  return pc;
}

bool call_trace_on(const cmtv_ctx* ctx) { return ctx->call_trace; }
uint64_t call_trace_now() { return now_ns_steady(); }
void call_trace_begin_locked(cmtv_ctx* ctx) { ctx->trace_launch = ctx->trace_wait = 0; }
void call_trace_record_locked(cmtv_ctx* ctx, uint64_t t_entry, uint64_t t_locked) {
  const uint64_t t_end = now_ns_steady();
  if (!ctx->trace_launch || !ctx->trace_wait) return;  // no small host batch ran
  if (ctx->call_trace_loaded_only && !ctx->bulk_now) return;
  std::lock_guard<std::mutex> g(ctx->trace_mu);
  ctx->trace_rows.push_back({t_locked - t_entry, ctx->trace_launch - t_locked, ctx->trace_wait - ctx->trace_launch,
                             t_end - ctx->trace_wait, ctx->trace_dev_ns});
}

void note_latency(cmtv_ctx* ctx) {
  ctx->last_latency_ns.store(now_ns_steady(), std::memory_order_relaxed);
}

bool latency_recent(const cmtv_ctx* ctx) {
  if (!ctx->lat_window_ns) return false;
  const uint64_t t = ctx->last_latency_ns.load(std::memory_order_relaxed);
  return t && now_ns_steady() - t < ctx->lat_window_ns;
}

LatencyStreams::LatencyStreams(cmtv_ctx* c) : ctx(c) {
  // the pipeline's masked chunks leave the reserved CUs free only while the
  // latency window is open; bulk_now (snapshotted at ctx_lock) says a
  // pipeline call is in flight
  if (!ctx->bulk_now || !ctx->lat_window_ns || !ctx->lat_isolate) return;
  for (size_t g : ctx->live) {
    CmtvDev& D = ctx->devs[g];
    BulkLane& L = D.bulk;
    if (!L.lat || D.failed || g >= 64) continue;
    (void)hipSetDevice(D.ordinal);
    // everything already on the normal stream (keyset builds, a polled
    // launch) completes first -- through an event only when something is
    // still in flight there: a cross-queue wait costs the launch ~45 us
    // (tools/lat_queue_probe.hip: 22.8 -> 69.2 us p50 for a 10 us kernel)
    const hipError_t q = hipStreamQuery(D.stream);
    if (q != hipSuccess && (q != hipErrorNotReady || hipEventRecord(L.lat_in, D.stream) != hipSuccess ||
                            hipStreamWaitEvent(L.lat, L.lat_in, 0) != hipSuccess)) {
      (void)hipGetLastError();
      continue;
    }
    std::swap(D.stream, L.lat);
    swapped |= 1ull << g;
  }
  if (swapped) ctx->stats.isolated_calls++;
  if (!ctx->live.empty()) (void)hipSetDevice(ctx->devs[ctx->live[0]].ordinal);
}

LatencyStreams::~LatencyStreams() {
  for (size_t g = 0; g < 64 && swapped; g++) {
    if (!(swapped >> g & 1)) continue;
    CmtvDev& D = ctx->devs[g];
    BulkLane& L = D.bulk;
    (void)hipSetDevice(D.ordinal);
    std::swap(D.stream, L.lat);
    // and what the call left in flight (a polled launch retiring) precedes
    // whatever comes next on the normal stream (an event only if needed)
    const hipError_t q = hipStreamQuery(L.lat);
    if (q == hipErrorNotReady) {
      if (hipEventRecord(L.lat_out, L.lat) != hipSuccess || hipStreamWaitEvent(D.stream, L.lat_out, 0) != hipSuccess)
        (void)hipGetLastError();
    } else if (q != hipSuccess) {
      (void)hipGetLastError();
    }
  }
  if (swapped && !ctx->live.empty()) (void)hipSetDevice(ctx->devs[ctx->live[0]].ordinal);
}

BulkBusy::BulkBusy(cmtv_ctx* c) : ctx(c) { ctx->bulk_busy.fetch_add(1, std::memory_order_relaxed); }
BulkBusy::~BulkBusy() { ctx->bulk_busy.fetch_sub(1, std::memory_order_relaxed); }

void live_devices_locked(cmtv_ctx* ctx, std::vector<size_t>& out) { out = ctx->live; }

static hipError_t bulk_lane_init(cmtv_ctx* ctx, CmtvDev& D) {
  BulkLane& L = D.bulk;
  if (L.exec) return hipSuccess;
  // Every stream of the lane gets a hardware queue of its own (a CU-masked
  // stream has one; plain streams share the process's GPU_MAX_HW_QUEUES
  // queues round-robin). On a shared queue the device's normal stream -- a
  // 150-validator VerifyCommit -- waits behind whatever the lane queued
  // before it: the barrier packet of an 80 MB chunk DMA, a 2.7 ms keyed
  // launch (round 6: p99 1.12 ms under a configs[2] load with the copy and
  // exec streams plain, bench latency_150_under_load).
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, D.ordinal);
  L.cus = (uint32_t)std::max(cus, 1);
  const uint32_t words = (L.cus + 31) / 32;
  std::vector<uint32_t> all(words, 0);
  for (uint32_t c = 0; c < L.cus; c++) all[c / 32] |= 1u << (c % 32);
  auto own_queue = [&](hipStream_t* st) {
    if (hipExtStreamCreateWithCUMask(st, words, all.data()) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
  };
  hipError_t e = own_queue(&L.copy);
  // CMTV_ONE_EXEC=1 (experiment): no unmasked exec queue -- every chunk on
  // the masked one (a queue fewer per lane, 16 CUs fewer for the bulk)
  if (e == hipSuccess && !ctx->one_exec) e = own_queue(&L.exec);

  if (e == hipSuccess) e = hipEventCreateWithFlags(&L.scratch.done, hipEventDisableTiming);
  if (e == hipSuccess) {
    // The reserved CUs: the masked exec stream gets every other CU, the
    // latency stream these. The driver deals a queue's CU-mask bits out
    // XCD-major round-robin -- bit i to XCD i mod 8, then to SE (i / 8) mod
    // 4, then to that SE's CU i / 32 (tools/cumask_probe.hip on MI355X:
    // bits 0..7 alone run on CU 0 of SE 0 of each XCD) -- and the dispatcher
    // deals a kernel's workgroups to the XCDs round-robin, so the reserve
    // must hold CUs on every XCD (an XCD whose share of a mask is empty runs
    // the queue on all its CUs). Taken in whole CU pairs (the pair shares
    // one instruction cache): bits 0..7 and 32..39 are CUs 0 and 1 of SE 0
    // on each XCD, then 8..15 and 40..47 (SE 1), and so on.
    std::vector<uint32_t> mask = all, lat(words, 0);
    const uint32_t reserved = reserved_cus(ctx, L.cus);
    for (uint32_t k = 0; k < reserved; k++) {
      const uint32_t pair = k / 16, cu_bit = (k / 8) % 2, xcd = k % 8;
      const uint32_t b = cu_bit * 32 + pair * 8 + xcd;
      mask[b / 32] &= ~(1u << (b % 32));
      lat[b / 32] |= 1u << (b % 32);
    }
    L.masked_waves = 8 * (L.cus - reserved);
    if (reserved == 0 || L.cus <= reserved ||
        hipExtStreamCreateWithCUMask(&L.exec_masked, words, mask.data()) != hipSuccess) {
      (void)hipGetLastError();
      L.exec_masked = nullptr;  // no masking: chunks keep the plain exec stream
    }
    if (L.exec_masked && ctx->lat_isolate) {
      if (hipExtStreamCreateWithCUMask(&L.lat, words, lat.data()) != hipSuccess ||
          hipEventCreateWithFlags(&L.lat_in, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&L.lat_out, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        if (L.lat) (void)hipStreamDestroy(L.lat);
        L.lat = nullptr;  // latency calls keep the normal stream
      }
    }
  }
  if (e == hipSuccess && !L.exec) {
    if (L.exec_masked)
      L.exec = L.exec_masked;
    else
      e = own_queue(&L.exec);
  }
  for (int k = 0; k < kBulkSlotsMax && e == hipSuccess; k++) {
    e = hipEventCreateWithFlags(&L.slot[k].h2d, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&L.slot[k].done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&L.slot[k].prep, hipEventDisableTiming);
  }
  (void)ctx;
  return e;
}

static void bulk_lane_release(CmtvDev& D) {
  BulkLane& L = D.bulk;
  if (L.exec) (void)hipStreamSynchronize(L.exec);
  if (L.exec_masked) (void)hipStreamSynchronize(L.exec_masked);
  if (L.copy) (void)hipStreamSynchronize(L.copy);
  if (L.prep) (void)hipStreamSynchronize(L.prep);
  for (auto& S : L.slot) {
    S.h_in.release();
    S.h_bm.release();
    S.d_in.release();
    S.d_bm.release();
    if (S.h2d) (void)hipEventDestroy(S.h2d);
    if (S.done) (void)hipEventDestroy(S.done);
    if (S.prep) (void)hipEventDestroy(S.prep);
    S.h2d = S.done = S.prep = nullptr;
    S.pending = false;
  }
  L.scratch.buf.release();
  if (L.scratch.done) (void)hipEventDestroy(L.scratch.done);
  L.scratch.done = nullptr;
  L.scratch.used = false;
  if (L.exec == L.exec_masked) L.exec = nullptr;  // CMTV_ONE_EXEC: one stream
  if (L.exec) (void)hipStreamDestroy(L.exec);
  if (L.exec_masked) (void)hipStreamDestroy(L.exec_masked);
  if (L.copy) (void)hipStreamDestroy(L.copy);
  if (L.lat) (void)hipStreamDestroy(L.lat);
  if (L.prep) (void)hipStreamDestroy(L.prep);
  L.prep = nullptr;
  if (L.lat_in) (void)hipEventDestroy(L.lat_in);
  if (L.lat_out) (void)hipEventDestroy(L.lat_out);
  L.exec = L.exec_masked = L.copy = L.lat = nullptr;
  L.lat_in = L.lat_out = nullptr;
}

int bulk_stage(cmtv_ctx* ctx, size_t dev, int slot, const BulkLayout& L, uint8_t** host) {
  CmtvDev& D = ctx->devs[dev];
  if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
  hipError_t e = bulk_lane_init(ctx, D);
  BulkSlot& S = D.bulk.slot[slot];
  if (e == hipSuccess) e = S.h_in.ensure(L.in_bytes);
  if (e != hipSuccess) return hip_fail(e);
  *host = static_cast<uint8_t*>(S.h_in.p);
  return CMTV_OK;
}

// Where a chunk's gather + sign-bytes run: an unmasked chunk's on the lane's
// masked exec stream -- idle while no latency call is near, and a queue the
// lane already has -- so they overlap the previous chunk's keyed launch on
// exec (VerifyCommit pass 39.9 -> 39.3 ms, profiles/r06_prep_stream_ab.txt);
// a masked chunk's in line on its own stream (CMTV_PREP_STREAM=0: always in
// line)
static hipStream_t bulk_prep_stream(const cmtv_ctx* ctx, const BulkLane& BL, bool masked) {
  if (masked) return BL.exec_masked;
  return ctx->prep_stream && BL.exec_masked ? BL.exec_masked : BL.exec;
}

int bulk_prepare(cmtv_ctx* ctx, size_t dev, int slot, const BulkLayout& L, const cmtv_keyset* ks) {
  // Everything of a chunk's submission that touches only the lane (its
  // streams, its slot's buffers): the staging's H2D, the direct chunk's
  // DMAs and gather, the sign-bytes. The bulk lock orders it; the context
  // lock is not taken, so a latency call never waits behind these ~10 HIP
  // calls (round 6) -- bulk_submit_locked then enqueues the launch.
  CmtvDev& D = ctx->devs[dev];
  if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
  BulkLane& BL = D.bulk;
  BulkSlot& S = BL.slot[slot];
  const size_t words = (L.m + 63) / 64;
  hipError_t e = S.d_in.ensure(L.dev_bytes);
  if (e == hipSuccess) e = S.d_bm.ensure(8 * std::max<size_t>(words, 1));
  if (e == hipSuccess) e = S.h_bm.ensure(8 * std::max<size_t>(words, 1));
  if (e != hipSuccess) return hip_fail(e);
  const bool masked = L.masked && BL.exec_masked;
  hipStream_t ex = masked ? BL.exec_masked : BL.exec;
  auto* din = static_cast<uint8_t*>(S.d_in.p);
  // H2D on the copy stream (overlaps the exec stream's previous chunk); a
  // direct chunk's per-signature data comes straight from the caller's
  // pinned arena, one DMA per span, and is laid out by k_bulk_gather
  if ((e = hipMemcpyAsync(din, S.h_in.p, L.in_bytes, hipMemcpyHostToDevice, BL.copy)) != hipSuccess) return hip_fail(e);
  if (L.direct)
    for (int k = 0; k < L.n_spans; k++)
      if ((e = hipMemcpyAsync(din + L.o_arena + L.spans[k].dev_off, L.spans[k].host, L.spans[k].bytes,
                              hipMemcpyHostToDevice, BL.copy)) != hipSuccess)
        return hip_fail(e);
  // the gather and the sign-bytes: on the prep stream for an unmasked chunk
  // (they overlap the previous chunk's keyed launch on exec: ~60 + 40 us a
  // chunk, round 6 rocprof of replay_c3_host), else in line on exec
  hipStream_t ps = bulk_prep_stream(ctx, BL, masked);
  if ((e = hipEventRecord(S.h2d, BL.copy)) != hipSuccess || (e = hipStreamWaitEvent(ps, S.h2d, 0)) != hipSuccess)
    return hip_fail(e);
  auto* off = reinterpret_cast<uint32_t*>(din + L.o_off);
  if (L.direct) {
    if (!ks) return CMTV_EINVAL;  // direct chunks are registered-key chunks
    auto* cb = reinterpret_cast<uint32_t*>(din + L.o_cbase);
    if ((e = launch_bulk_gather((uint32_t)L.n_tmpls, (uint32_t)L.m, din + L.o_desc, din + L.o_tmpl, din + L.o_arena,
                                reinterpret_cast<uint32_t*>(din + L.o_key), din + L.o_sig, off,
                                reinterpret_cast<uint32_t*>(din + L.o_tidx), din + L.o_flag,
                                reinterpret_cast<int64_t*>(din + L.o_sec), reinterpret_cast<int32_t*>(din + L.o_nanos),
                                cb, cb + L.n_tmpls, ps)) != hipSuccess)
      return hip_fail(e);
  }
  // sign-bytes from the chunk's templates into o_msg (k_sign_bytes; the
  // bulk chunks run the lane kernels, whose launches take no fused form)
  if ((e = launch_sign_bytes((uint32_t)L.m, din + L.o_tmpl, din + L.o_blob, reinterpret_cast<uint32_t*>(din + L.o_tidx),
                             din + L.o_flag, reinterpret_cast<int64_t*>(din + L.o_sec),
                             reinterpret_cast<int32_t*>(din + L.o_nanos), off, din + L.o_msg, ps)) != hipSuccess)
    return hip_fail(e);
  if (ps != ex && (e = hipEventRecord(S.prep, ps)) != hipSuccess) return hip_fail(e);
  return CMTV_OK;
}

int bulk_submit_locked(cmtv_ctx* ctx, size_t dev, int slot, const BulkLayout& L, const cmtv_keyset* ks,
                       uint32_t mode) {
  CmtvDev& D = ctx->devs[dev];
  if (D.failed) return CMTV_EHIP;  // retired by another call meanwhile
  if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
  BulkLane& BL = D.bulk;
  BulkSlot& S = BL.slot[slot];
  const size_t words = (L.m + 63) / 64;
  hipError_t e;
  // near a latency call: the CU-masked stream, and batched launches sized
  // to the waves its CUs hold in one round
  const bool masked = L.masked && BL.exec_masked;
  hipStream_t ex = masked ? BL.exec_masked : BL.exec;
  auto* din = static_cast<uint8_t*>(S.d_in.p);
  auto* dbm = static_cast<uint64_t*>(S.d_bm.p);
  auto* off = reinterpret_cast<uint32_t*>(din + L.o_off);
  // the chunk's prep (bulk_prepare) ran on the prep stream: exec waits for it
  if (bulk_prep_stream(ctx, BL, masked) != ex && (e = hipStreamWaitEvent(ex, S.prep, 0)) != hipSuccess)
    return hip_fail(e);
  int rc;
  // a registered-key chunk's kernel stores its verdict words straight into
  // the slot's mapped host bitmap: no D2H between this launch and the next
  // chunk's on exec (round 6: consecutive keyed launches were 84-135 us
  // apart, ~2 ms of a 40 ms pass; CMTV_BULK_BM_DIRECT=1, measured neutral)
  uint64_t* hbm_dev = nullptr;
  if (ks && ctx->bulk_bm_direct) {
    void* q = nullptr;
    if ((e = hipHostGetDevicePointer(&q, S.h_bm.p, 0)) != hipSuccess) return hip_fail(e);
    hbm_dev = static_cast<uint64_t*>(q);
  }
  if (ks)
    rc = enqueue_verify_keyed(ctx, D, ks->dev[dev], ks->n, L.m, reinterpret_cast<uint32_t*>(din + L.o_key),
                              din + L.o_sig, din + L.o_msg, off, mode, nullptr, hbm_dev ? hbm_dev : dbm, ex,
                              &BL.scratch, nullptr, masked ? BL.masked_waves : 0);
  else
    rc = enqueue_verify(ctx, D, L.m, din + L.o_key, din + L.o_sig, din + L.o_msg, off, mode, nullptr, dbm, ex,
                        nullptr, &BL.scratch);
  if (rc != CMTV_OK) return rc;
  if ((!hbm_dev && (e = hipMemcpyAsync(S.h_bm.p, dbm, 8 * words, hipMemcpyDeviceToHost, ex)) != hipSuccess) ||
      (e = hipEventRecord(S.done, ex)) != hipSuccess)
    return hip_fail(e);
  S.pending = true;
  if (masked) ctx->stats.masked_chunks++;
  return CMTV_OK;
}

int bulk_wait(cmtv_ctx* ctx, size_t dev, int slot, const uint64_t** bitmap) {
  CmtvDev& D = ctx->devs[dev];
  BulkSlot& S = D.bulk.slot[slot];
  if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
  const hipError_t e = hipEventSynchronize(S.done);
  S.pending = false;
  if (e != hipSuccess) return hip_fail(e);
  if ((long)dev == ctx->fault_sync_dev) return CMTV_EHIP;  // CMTV_FAULT_SYNC_DEV (see run_host_batch_)
  *bitmap = static_cast<const uint64_t*>(S.h_bm.p);
  return CMTV_OK;
}

void bulk_drain(cmtv_ctx* ctx) {
  for (auto& D : ctx->devs) {
    if (!D.bulk.exec) continue;
    (void)hipSetDevice(D.ordinal);
    (void)hipStreamSynchronize(D.bulk.copy);
    (void)hipStreamSynchronize(D.bulk.exec);
    if (D.bulk.exec_masked) (void)hipStreamSynchronize(D.bulk.exec_masked);
    if (D.bulk.prep) (void)hipStreamSynchronize(D.bulk.prep);
    for (auto& S : D.bulk.slot) S.pending = false;
  }
  (void)hipGetLastError();
}

bool retire_device_locked(cmtv_ctx* ctx, size_t dev) {
  // retired meanwhile by another call (the pipeline holds the lock only
  // around submissions): already out of the rotation, so the chunks run again
  // on whatever is still live
  if (ctx->devs[dev].failed) return !ctx->live.empty();
  // CMTV_FAULT_AT stands for a failure of the call, not of the device
  const bool injected = ctx->fault_pending;
  ctx->fault_pending = false;
  if (injected || ctx->live.size() < 2) return false;
  retire_device(ctx, dev);
  ctx->stats.reshards++;
  return true;
}

void count_invalid_locked(cmtv_ctx* ctx, uint64_t n) { ctx->stats.invalid += n; }
void count_direct_locked(cmtv_ctx* ctx) { ctx->stats.direct_chunks++; }

bool pinned_holds_locked(const cmtv_ctx* ctx, const void* p, size_t bytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = ctx->pinned.upper_bound(a);
  if (it == ctx->pinned.begin()) return false;
  --it;
  return a + bytes >= a && a + bytes <= it->first + it->second;
}

void pinned_ranges_locked(cmtv_ctx* ctx, std::vector<PinnedRange>& out) {
  out.clear();
  for (auto& b : ctx->pinned) out.push_back(PinnedRange{b.first, b.second});
}

PipeWorkspace*& pipe_workspace(cmtv_ctx* ctx) { return ctx->pipe_ws; }

}  // namespace cmtv

extern "C" {

int cmtv_alloc_pinned(cmtv_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out || bytes == 0) return CMTV_EINVAL;
  *out = nullptr;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  void* p = nullptr;
  // portable: every device of the context DMAs from it
  if (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess || !p) {
    (void)hipGetLastError();
    return CMTV_ENOMEM;
  }
  try {
    ctx->pinned.emplace(reinterpret_cast<uintptr_t>(p), bytes);
  } catch (...) {
    (void)hipHostFree(p);
    return CMTV_ENOMEM;
  }
  *out = p;
  return CMTV_OK;
}

int cmtv_free_pinned(cmtv_ctx* ctx, void* p) {
  if (!ctx) return CMTV_EINVAL;
  if (!p) return CMTV_OK;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  auto it = ctx->pinned.find(reinterpret_cast<uintptr_t>(p));
  if (it == ctx->pinned.end()) return CMTV_EINVAL;  // not this context's block
  ctx->pinned.erase(it);
  return hipHostFree(p) == hipSuccess ? CMTV_OK : CMTV_EHIP;
}

void cmtv_keyset_free(cmtv_keyset* ks) {
  if (!ks) return;
  for (size_t g = 0; g < ks->dev.size(); g++) {
    (void)hipSetDevice(ks->ctx->devs[g].ordinal);
    (void)hipStreamSynchronize(ks->ctx->devs[g].stream);  // no kernel may still read the combs
    auto& K = ks->dev[g];
    if (K.d_pk) (void)hipFree(K.d_pk);
    if (K.d_ok) (void)hipFree(K.d_ok);
    if (K.d_tab) (void)hipFree(K.d_tab);
    if (K.d_wide) (void)hipFree(K.d_wide);
  }
  if (!ks->ctx->devs.empty()) (void)hipSetDevice(ks->ctx->devs[0].ordinal);
  delete ks;
}

size_t cmtv_keyset_len(const cmtv_keyset* ks) { return ks ? ks->n : 0; }

int cmtv_verify_ed25519_indexed(cmtv_ctx* ctx, const cmtv_keyset* ks, size_t n, const uint32_t* key_idx,
                                const uint8_t* sig, const uint8_t* msg, const uint32_t* msg_off, uint32_t mode,
                                uint8_t* out_valid, uint64_t* out_bitmap) {
  if (!ctx || !ks || ks->ctx != ctx || mode > CMTV_MODE_ZIP215 || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!key_idx || !sig || !msg_off || (!msg && msg_off[n] != 0) || (!out_valid && !out_bitmap)) return CMTV_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (msg_off[i + 1] < msg_off[i] || key_idx[i] >= ks->n) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  static const uint8_t empty = 0;
  HostBatch B;
  B.n = n;
  B.mode = mode;
  B.ks = ks;
  B.key_idx = key_idx;
  B.sig = sig;
  B.msg = msg ? msg : &empty;
  B.msg_off = msg_off;
  return run_host_batch(ctx, B, out_valid, out_bitmap);
}

int cmtv_verify_ed25519_indexed_device(cmtv_ctx* ctx, const cmtv_keyset* ks, size_t n, const void* d_key_idx,
                                       const void* d_sig, const void* d_msg, const void* d_msg_off, uint32_t mode,
                                       void* d_valid, void* d_bitmap, void* stream) {
  if (!ctx || !ks || ks->ctx != ctx || mode > CMTV_MODE_ZIP215 || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!d_key_idx || !d_sig || !d_msg || !d_msg_off || (!d_valid && !d_bitmap)) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  if (dev0_usable(ctx) != CMTV_OK) return CMTV_ENODEV;
  // a key set registered after device 0 was retired has no tables there
  if (!ks->dev[0].d_tab || !ks->dev[0].d_pk || !ks->dev[0].d_ok) return CMTV_ENODEV;
  return single_device_rc(
      ctx, enqueue_verify_keyed(ctx, ctx->devs[0], ks->dev[0], ks->n, n, static_cast<const uint32_t*>(d_key_idx),
                                static_cast<const uint8_t*>(d_sig), static_cast<const uint8_t*>(d_msg),
                                static_cast<const uint32_t*>(d_msg_off), mode, static_cast<uint8_t*>(d_valid),
                                static_cast<uint64_t*>(d_bitmap), static_cast<hipStream_t>(stream)));
}

int cmtv_pubkeys_ed25519(cmtv_ctx* ctx, size_t n, const uint8_t* seeds, uint8_t* out_pk) {
  if (!ctx || n > (1ull << 31) || (n && (!seeds || !out_pk))) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  // host buffers in and out: the first live device does it
  if (ctx->live.empty()) return CMTV_ENODEV;
  CmtvDev& D = ctx->devs[ctx->live[0]];
  if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
  hipError_t e;
  if ((e = D.d_in.ensure(32 * n)) != hipSuccess) return hip_fail(e);
  if ((e = D.d_out.ensure(32 * n)) != hipSuccess) return hip_fail(e);
  if ((e = hipMemcpyAsync(D.d_in.p, seeds, 32 * n, hipMemcpyHostToDevice, D.stream)) != hipSuccess)
    return hip_fail(e);
  for (size_t c = 0; c < n; c += kChunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(kChunk, n - c);
    if ((e = launch_pubkey(cn, static_cast<uint8_t*>(D.d_in.p) + 32 * c, D.d_btab,
                           static_cast<uint8_t*>(D.d_out.p) + 32 * c, D.stream)) != hipSuccess)
      return hip_fail(e);
  }
  if ((e = hipMemcpyAsync(out_pk, D.d_out.p, 32 * n, hipMemcpyDeviceToHost, D.stream)) != hipSuccess)
    return hip_fail(e);
  if ((e = hipStreamSynchronize(D.stream)) != hipSuccess) return hip_fail(e);
  return CMTV_OK;
}

int cmtv_sign_ed25519(cmtv_ctx* ctx, size_t n, const uint8_t* seeds, const uint32_t* key_idx, const uint8_t* msg,
                      const uint32_t* msg_off, uint8_t* out_sig) {
  if (!ctx || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!seeds || !msg_off || !out_sig || (!msg && msg_off[n] != 0)) return CMTV_EINVAL;
  size_t nseeds = n;
  if (key_idx) {
    nseeds = 0;
    for (size_t i = 0; i < n; i++) nseeds = std::max<size_t>(nseeds, (size_t)key_idx[i] + 1);
  }
  for (size_t i = 0; i < n; i++)
    if (msg_off[i + 1] < msg_off[i]) return CMTV_EINVAL;
  std::unique_lock<std::mutex> lk;
  if (ctx_lock(ctx, lk) != CMTV_OK) return CMTV_ENODEV;
  // host buffers in and out: the first live device does it
  if (ctx->live.empty()) return CMTV_ENODEV;
  CmtvDev& D = ctx->devs[ctx->live[0]];
  if (hipSetDevice(D.ordinal) != hipSuccess) return CMTV_ENODEV;
  const size_t msg_bytes = msg_off[n];
  const size_t o_seed = 0, o_idx = align_up(32 * nseeds, 256), o_off = align_up(o_idx + (key_idx ? 4 * n : 0), 256);
  const size_t o_msg = align_up(o_off + 4 * (n + 1), 256), in_bytes = align_up(o_msg + msg_bytes + 16, 256);
  hipError_t e;
  if ((e = D.h_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = D.d_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = D.d_out.ensure(64 * n)) != hipSuccess) return hip_fail(e);
  auto* hin = static_cast<uint8_t*>(D.h_in.p);
  std::memcpy(hin + o_seed, seeds, 32 * nseeds);
  if (key_idx) std::memcpy(hin + o_idx, key_idx, 4 * n);
  std::memcpy(hin + o_off, msg_off, 4 * (n + 1));
  if (msg_bytes) std::memcpy(hin + o_msg, msg, msg_bytes);
  auto* din = static_cast<uint8_t*>(D.d_in.p);
  if ((e = hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, D.stream)) != hipSuccess) return hip_fail(e);
  for (size_t c = 0; c < n; c += kChunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(kChunk, n - c);
    if ((e = launch_sign(cn, key_idx ? din + o_seed : din + o_seed + 32 * c, key_idx ? din + o_idx + 4 * c : nullptr,
                         din + o_msg, din + o_off + 4 * c, D.d_btab, static_cast<uint8_t*>(D.d_out.p) + 64 * c,
                         D.stream)) != hipSuccess)
      return hip_fail(e);
  }
  if ((e = hipMemcpyAsync(out_sig, D.d_out.p, 64 * n, hipMemcpyDeviceToHost, D.stream)) != hipSuccess)
    return hip_fail(e);
  if ((e = hipStreamSynchronize(D.stream)) != hipSuccess) return hip_fail(e);
  return CMTV_OK;
}

}  // extern "C"
