// runtime.cpp -- libcmtverify host runtime: contexts, streams, pinned staging,
// chunked kernel launches and the C ABI of include/cmtverify.h.
//
// One context = one device + one HIP stream + the device-resident fixed-base
// table + growable device/pinned buffers. Calls on a context are serialised
// by its mutex and start with hipSetDevice (cgo callers migrate threads).
// There is no CPU verification path: if the device is unusable every call
// fails with a negative code and the caller decides what to do.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/cmtverify.h"
#include "kernels.h"
#include "merlin.h"
#include "signbytes.h"
#include "runtime_internal.h"

namespace {

constexpr uint32_t kChunk = 1u << 18;  // signatures per launch (A-table scratch = kChunk * 1280 B)
// crossover between the quad (4 lanes / signature) and lane (1 lane / signature)
// kernels; measured on MI355X, overridable with CMTV_QUAD_MAX
constexpr size_t kQuadMaxDefault = 40000;
// the same crossover for registered-key verification (env CMTV_KEYED_QUAD_MAX)
constexpr size_t kKeyedQuadMaxDefault = 16384;

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
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    want = want + want / 4;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Verdict cache (cmtv_verdict_cache): a ring of the last `cap` verdicts,
// indexed by a 64-bit hash of (mode, signature); a hit also compares the full
// key bytes (mode, pk, sig, msg), so it returns exactly the device verdict.
struct VerdictCache {
  struct Entry {
    std::string key;
    uint64_t h = 0;
    uint8_t verdict = 0;
    bool used = false;
  };
  size_t cap = 0;
  size_t next = 0;
  std::vector<Entry> ring;
  std::unordered_multimap<uint64_t, size_t> index;

  static uint64_t hash(uint32_t mode, const uint8_t* sig) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ mode;
    for (int i = 0; i < 8; i++) {
      uint64_t w;
      std::memcpy(&w, sig + 8 * i, 8);
      h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
      h ^= h >> 31;
    }
    return h;
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

}  // namespace

struct cmtv_ctx {
  int device = 0;
  uint32_t default_mode = CMTV_MODE_GO_STDLIB;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timing_pending = false;
  uint32_t* d_btab = nullptr;
  DevBuf d_atab, d_in, d_out;
  HostBuf h_in, h_out;
  std::mutex mu;
  cmtv_stats stats{};
  size_t quad_max = kQuadMaxDefault;  // batches up to this size use the quad kernel
  uint32_t* d_bcomb = nullptr;        // comb of B for registered-key verification (built lazily)
  uint16_t* d_srprog = nullptr;       // sr25519 transcript program (merlin.h)
  int sr_nops = 0;
  VerdictCache cache;                 // cmtv_verdict_cache (off by default)
  size_t lane_chunk = kChunk;         // signatures per lane-kernel launch (env CMTV_LANE_CHUNK)
  size_t keyed_quad_max = kKeyedQuadMaxDefault;  // registered-key batches up to this use the quad kernel
  // cmtv_keyset_cache: validator sets (their concatenated keys) -> registered
  // key sets, used by cmtv_verify_commit(s); FIFO of at most keyset_cap
  size_t keyset_cap = 0;
  std::vector<std::pair<std::string, cmtv_keyset*>> keysets;
};

struct cmtv_keyset {
  cmtv_ctx* ctx = nullptr;
  size_t n = 0;
  uint32_t* d_pk = nullptr;   // n x 8 words, the keys' original bytes
  uint8_t* d_ok = nullptr;    // n decode flags
  uint32_t* d_tab = nullptr;  // n x kCombWords
  std::vector<uint8_t> pk;    // host copy (n x 32)
};

namespace cmtv {

static int hip_fail(hipError_t e) {
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return CMTV_ENOMEM;
  return CMTV_EHIP;
}

static void harvest_timing(cmtv_ctx* ctx) {
  if (!ctx->timing_pending) return;
  if (hipEventSynchronize(ctx->ev1) == hipSuccess) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) == hipSuccess) {
      ctx->stats.last_kernel_ms = ms;
      ctx->stats.device_ms += ms;
    }
  }
  ctx->timing_pending = false;
}

// Enqueue verification of n signatures whose inputs are in device memory.
static int enqueue_verify(cmtv_ctx* ctx, size_t n, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                          const uint32_t* d_off, uint32_t mode, uint8_t* d_valid, uint64_t* d_bitmap,
                          hipStream_t s) {
  if (n == 0) return CMTV_OK;
  // Small batches cannot fill the chip at one signature per lane: use the
  // 4-lanes-per-signature kernel below the crossover (quad.h,
  // sr25519_quad.h).
  const bool sr = mode == kModeSr25519;
  const bool quad = n <= ctx->quad_max;
  hipError_t e = hipSuccess;
  if (!quad) {
    const size_t lanes = std::min<size_t>(n, ctx->lane_chunk);
    const size_t lanes_padded = (lanes + 63) / 64 * 64;
    e = ctx->d_atab.ensure(lanes_padded * kAtabWordsPerLane * sizeof(uint32_t));
    if (e != hipSuccess) return hip_fail(e);
  }
  harvest_timing(ctx);
  if ((e = hipEventRecord(ctx->ev0, s)) != hipSuccess) return hip_fail(e);
  const size_t chunk = quad ? kChunk : ctx->lane_chunk;
  for (size_t c = 0; c < n; c += chunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(chunk, n - c);
    if (sr)
      e = launch_verify_sr25519(cn, d_pk + 32 * c, d_sig + 64 * c, d_msg, d_off + c, ctx->d_btab,
                                static_cast<uint32_t*>(ctx->d_atab.p), ctx->d_srprog, ctx->sr_nops,
                                d_valid ? d_valid + c : nullptr, d_bitmap ? d_bitmap + c / 64 : nullptr, quad, s);
    else
      e = launch_verify(mode, cn, d_pk + 32 * c, d_sig + 64 * c, d_msg, d_off + c, ctx->d_btab,
                        static_cast<uint32_t*>(ctx->d_atab.p), d_valid ? d_valid + c : nullptr,
                        d_bitmap ? d_bitmap + c / 64 : nullptr, quad, s);
    if (e != hipSuccess) return hip_fail(e);
    ctx->stats.kernel_launches++;
  }
  if ((e = hipEventRecord(ctx->ev1, s)) != hipSuccess) return hip_fail(e);
  ctx->timing_pending = true;
  ctx->stats.calls++;
  ctx->stats.signatures += n;
  return CMTV_OK;
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// keys per comb-build launch (prefix-product scratch = 160 KiB per key)
constexpr uint32_t kCombKeyChunk = 256;

// Comb of B (keyed.h), built on first use; caller holds the context lock.
static int ensure_bcomb(cmtv_ctx* ctx) {
  if (ctx->d_bcomb) return CMTV_OK;
  const uint32_t bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  DevBuf scratch, bpk;
  uint32_t* tab = nullptr;
  hipError_t e = hipMalloc(&tab, kCombWords * sizeof(uint32_t));
  if (e == hipSuccess) e = scratch.ensure(kCombScratchWordsPerKey * sizeof(uint32_t));
  if (e == hipSuccess) e = bpk.ensure(sizeof(bw));
  if (e == hipSuccess) e = hipMemcpyAsync(bpk.p, bw, sizeof(bw), hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess)
    e = launch_comb_build(1, bpk.p, nullptr, tab, static_cast<uint32_t*>(scratch.p), false, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  scratch.release();
  bpk.release();
  if (e != hipSuccess) {
    if (tab) (void)hipFree(tab);
    return hip_fail(e);
  }
  ctx->d_bcomb = tab;
  return CMTV_OK;
}

static int enqueue_verify_keyed(cmtv_ctx* ctx, const cmtv_keyset* ks, size_t n, const uint32_t* d_idx,
                                const uint8_t* d_sig, const uint8_t* d_msg, const uint32_t* d_off, uint32_t mode,
                                uint8_t* d_valid, uint64_t* d_bitmap, hipStream_t s) {
  if (n == 0) return CMTV_OK;
  harvest_timing(ctx);
  hipError_t e;
  if ((e = hipEventRecord(ctx->ev0, s)) != hipSuccess) return hip_fail(e);
  for (size_t c = 0; c < n; c += kChunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(kChunk, n - c);
    e = launch_verify_keyed(mode, cn, (uint32_t)ks->n, d_idx + c, d_sig + 64 * c, d_msg, d_off + c, ks->d_pk,
                            ks->d_ok, ks->d_tab, ctx->d_bcomb, d_valid ? d_valid + c : nullptr,
                            d_bitmap ? d_bitmap + c / 64 : nullptr, n <= ctx->keyed_quad_max, s);
    if (e != hipSuccess) return hip_fail(e);
    ctx->stats.kernel_launches++;
  }
  if ((e = hipEventRecord(ctx->ev1, s)) != hipSuccess) return hip_fail(e);
  ctx->timing_pending = true;
  ctx->stats.calls++;
  ctx->stats.signatures += n;
  return CMTV_OK;
}

static int verify_host_device(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                              const uint32_t* msg_off, uint32_t mode, uint8_t* out_valid, uint64_t* out_bitmap);

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
    hs[i] = VerdictCache::hash(mode, sig + 64 * i);
    VerdictCache::make_key(keys[i], mode, pk + 32 * i, sig + 64 * i, msg + msg_off[i], msg_off[i + 1] - msg_off[i]);
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

static int verify_host_device(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                              const uint32_t* msg_off, uint32_t mode, uint8_t* out_valid, uint64_t* out_bitmap) {
  if (n == 0) return CMTV_OK;
  const size_t msg_bytes = msg_off[n];
  // staging layout: [pk n*32][sig n*64][off (n+1)*4][msg msg_bytes + 16]
  const size_t o_pk = 0, o_sig = align_up(o_pk + 32 * n, 256), o_off = align_up(o_sig + 64 * n, 256);
  const size_t o_msg = align_up(o_off + 4 * (n + 1), 256), in_bytes = align_up(o_msg + msg_bytes + 16, 256);
  const size_t words = (n + 63) / 64;
  const size_t o_bm = 0, o_valid = align_up(8 * words, 256), out_bytes = align_up(o_valid + n, 256);
  hipError_t e;
  if ((e = ctx->h_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->h_out.ensure(out_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_out.ensure(out_bytes)) != hipSuccess) return hip_fail(e);
  auto* hin = static_cast<uint8_t*>(ctx->h_in.p);
  std::memcpy(hin + o_pk, pk, 32 * n);
  std::memcpy(hin + o_sig, sig, 64 * n);
  std::memcpy(hin + o_off, msg_off, 4 * (n + 1));
  if (msg_bytes) std::memcpy(hin + o_msg, msg, msg_bytes);
  std::memset(hin + o_msg + msg_bytes, 0, 16);
  auto* din = static_cast<uint8_t*>(ctx->d_in.p);
  auto* dout = static_cast<uint8_t*>(ctx->d_out.p);
  if ((e = hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess) return hip_fail(e);
  int rc = enqueue_verify(ctx, n, din + o_pk, din + o_sig, din + o_msg, reinterpret_cast<uint32_t*>(din + o_off), mode,
                          dout + o_valid, reinterpret_cast<uint64_t*>(dout + o_bm), ctx->stream);
  if (rc != CMTV_OK) return rc;
  auto* hout = static_cast<uint8_t*>(ctx->h_out.p);
  if ((e = hipMemcpyAsync(hout, dout, out_bytes, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess) return hip_fail(e);
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e);
  harvest_timing(ctx);
  uint64_t invalid = 0;
  const uint8_t* hv = hout + o_valid;
  for (size_t i = 0; i < n; i++) invalid += hv[i] == 0;
  ctx->stats.invalid += invalid;
  if (out_valid) std::memcpy(out_valid, hv, n);
  if (out_bitmap) std::memcpy(out_bitmap, hout + o_bm, 8 * words);
  return CMTV_OK;
}

int verify_templated_locked(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint32_t* msg_off,
                            const void* tmpls, size_t n_tmpls, const uint8_t* blob, size_t blob_len,
                            const uint32_t* tidx, const uint8_t* commit_flag, const int64_t* sec,
                            const int32_t* nanos, uint32_t mode, uint8_t* out_valid, const cmtv_keyset* ks,
                            const uint32_t* key_idx) {
  if (n == 0) return CMTV_OK;
  const size_t msg_bytes = msg_off[n];
  const size_t tb = n_tmpls * sizeof(SbTemplate);
  // staging: [pk][sig][off][tidx][flag][sec][nanos][templates][blob] | device only: [msg]
  const size_t o_pk = 0, o_sig = align_up(32 * n, 256), o_off = align_up(o_sig + 64 * n, 256);
  const size_t o_tidx = align_up(o_off + 4 * (n + 1), 256), o_flag = align_up(o_tidx + 4 * n, 256);
  const size_t o_sec = align_up(o_flag + n, 256), o_nanos = align_up(o_sec + 8 * n, 256);
  const size_t o_tmpl = align_up(o_nanos + 4 * n, 256), o_blob = align_up(o_tmpl + tb, 256);
  const size_t in_bytes = align_up(o_blob + blob_len + 16, 256);
  const size_t o_msg = in_bytes, dev_bytes = align_up(o_msg + msg_bytes + 16, 256);
  const size_t o_valid = 0, out_bytes = align_up(n, 256);
  hipError_t e;
  if ((e = ctx->h_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_in.ensure(dev_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->h_out.ensure(out_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_out.ensure(out_bytes)) != hipSuccess) return hip_fail(e);
  auto* hin = static_cast<uint8_t*>(ctx->h_in.p);
  if (ks)
    std::memcpy(hin + o_pk, key_idx, 4 * n);  // key indices in the key slot
  else
    std::memcpy(hin + o_pk, pk, 32 * n);
  std::memcpy(hin + o_sig, sig, 64 * n);
  std::memcpy(hin + o_off, msg_off, 4 * (n + 1));
  std::memcpy(hin + o_tidx, tidx, 4 * n);
  std::memcpy(hin + o_flag, commit_flag, n);
  std::memcpy(hin + o_sec, sec, 8 * n);
  std::memcpy(hin + o_nanos, nanos, 4 * n);
  std::memcpy(hin + o_tmpl, tmpls, tb);
  if (blob_len) std::memcpy(hin + o_blob, blob, blob_len);
  auto* din = static_cast<uint8_t*>(ctx->d_in.p);
  auto* dout = static_cast<uint8_t*>(ctx->d_out.p);
  if ((e = hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess) return hip_fail(e);
  if ((e = hipMemsetAsync(din + o_msg + msg_bytes, 0, 16, ctx->stream)) != hipSuccess) return hip_fail(e);
  if ((e = launch_sign_bytes((uint32_t)n, din + o_tmpl, din + o_blob, reinterpret_cast<uint32_t*>(din + o_tidx),
                             din + o_flag, reinterpret_cast<int64_t*>(din + o_sec),
                             reinterpret_cast<int32_t*>(din + o_nanos), reinterpret_cast<uint32_t*>(din + o_off),
                             din + o_msg, ctx->stream)) != hipSuccess)
    return hip_fail(e);
  int rc = ks ? enqueue_verify_keyed(ctx, ks, n, reinterpret_cast<uint32_t*>(din + o_pk), din + o_sig, din + o_msg,
                                     reinterpret_cast<uint32_t*>(din + o_off), mode, dout + o_valid, nullptr,
                                     ctx->stream)
              : enqueue_verify(ctx, n, din + o_pk, din + o_sig, din + o_msg, reinterpret_cast<uint32_t*>(din + o_off),
                               mode, dout + o_valid, nullptr, ctx->stream);
  if (rc != CMTV_OK) return rc;
  auto* hout = static_cast<uint8_t*>(ctx->h_out.p);
  if ((e = hipMemcpyAsync(hout, dout, out_bytes, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess) return hip_fail(e);
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e);
  harvest_timing(ctx);
  uint64_t invalid = 0;
  for (size_t i = 0; i < n; i++) invalid += hout[o_valid + i] == 0;
  ctx->stats.invalid += invalid;
  std::memcpy(out_valid, hout + o_valid, n);
  return CMTV_OK;
}

int ctx_lock(cmtv_ctx* ctx, std::unique_lock<std::mutex>& lk) {
  lk = std::unique_lock<std::mutex>(ctx->mu);
  return hipSetDevice(ctx->device) == hipSuccess ? CMTV_OK : CMTV_ENODEV;
}

uint32_t ctx_default_mode(const cmtv_ctx* ctx) { return ctx->default_mode; }

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
  if (dev >= ndev) return CMTV_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return CMTV_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CMTV_ENODEV;
  if (hipSetDevice(dev) != hipSuccess) return CMTV_ENODEV;
  auto* ctx = new (std::nothrow) cmtv_ctx();
  if (!ctx) return CMTV_ENOMEM;
  ctx->device = dev;
  ctx->default_mode = cfg ? cfg->default_mode : CMTV_MODE_GO_STDLIB;
  if (const char* qm = std::getenv("CMTV_QUAD_MAX")) ctx->quad_max = (size_t)std::strtoull(qm, nullptr, 10);
  if (const char* kq = std::getenv("CMTV_KEYED_QUAD_MAX")) ctx->keyed_quad_max = (size_t)std::strtoull(kq, nullptr, 10);
  if (const char* lc = std::getenv("CMTV_LANE_CHUNK")) {
    const size_t v = (size_t)std::strtoull(lc, nullptr, 10) / 64 * 64;
    if (v >= 64 && v <= kChunk) ctx->lane_chunk = v;
  }
  hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev0);
  if (e == hipSuccess) e = hipEventCreate(&ctx->ev1);
  if (e == hipSuccess) e = hipMalloc(&ctx->d_btab, kBtabWords * sizeof(uint32_t));
  if (e == hipSuccess) e = launch_btab_init(ctx->d_btab, ctx->stream);
  uint16_t prog[SR_PROGRAM_MAX];
  ctx->sr_nops = sr_build_program(prog);
  if (e == hipSuccess) e = hipMalloc(&ctx->d_srprog, sizeof(prog));
  if (e == hipSuccess) e = hipMemcpyAsync(ctx->d_srprog, prog, sizeof(prog), hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    cmtv_close(ctx);
    return hip_fail(e);
  }
  *out = ctx;
  return CMTV_OK;
}

void cmtv_close(cmtv_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  ctx->d_atab.release();
  ctx->d_in.release();
  ctx->d_out.release();
  ctx->h_in.release();
  ctx->h_out.release();
  if (ctx->d_btab) (void)hipFree(ctx->d_btab);
  if (ctx->d_bcomb) (void)hipFree(ctx->d_bcomb);
  if (ctx->d_srprog) (void)hipFree(ctx->d_srprog);
  for (auto& e : ctx->keysets) cmtv_keyset_free(e.second);
  ctx->keysets.clear();
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

void* cmtv_stream(cmtv_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

int cmtv_stats_get(cmtv_ctx* ctx, cmtv_stats* out) {
  if (!ctx || !out) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  harvest_timing(ctx);
  ctx->stats.cache_entries = ctx->cache.size();
  *out = ctx->stats;
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
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  return verify_host_locked(ctx, n, pk, sig, msg, msg_off, mode, out_valid, out_bitmap);
}

int cmtv_verify_ed25519_device(cmtv_ctx* ctx, size_t n, const void* d_pk, const void* d_sig, const void* d_msg,
                               const void* d_msg_off, uint32_t mode, void* d_valid, void* d_bitmap, void* stream) {
  if (!ctx || mode > CMTV_MODE_ZIP215 || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!d_pk || !d_sig || !d_msg || !d_msg_off || (!d_valid && !d_bitmap)) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
  return enqueue_verify(ctx, n, static_cast<const uint8_t*>(d_pk), static_cast<const uint8_t*>(d_sig),
                        static_cast<const uint8_t*>(d_msg), static_cast<const uint32_t*>(d_msg_off), mode,
                        static_cast<uint8_t*>(d_valid), static_cast<uint64_t*>(d_bitmap), s);
}

int cmtv_verify_sr25519(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                        const uint32_t* msg_off, uint8_t* out_valid, uint64_t* out_bitmap) {
  if (!ctx || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!pk || !sig || !msg_off || (!msg && msg_off[n] != 0) || (!out_valid && !out_bitmap)) return CMTV_EINVAL;
  for (size_t i = 0; i < n; i++)
    if (msg_off[i + 1] < msg_off[i]) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  return verify_host_locked(ctx, n, pk, sig, msg, msg_off, kModeSr25519, out_valid, out_bitmap);
}

int cmtv_verify_sr25519_device(cmtv_ctx* ctx, size_t n, const void* d_pk, const void* d_sig, const void* d_msg,
                               const void* d_msg_off, void* d_valid, void* d_bitmap, void* stream) {
  if (!ctx || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!d_pk || !d_sig || !d_msg || !d_msg_off || (!d_valid && !d_bitmap)) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  return enqueue_verify(ctx, n, static_cast<const uint8_t*>(d_pk), static_cast<const uint8_t*>(d_sig),
                        static_cast<const uint8_t*>(d_msg), static_cast<const uint32_t*>(d_msg_off), kModeSr25519,
                        static_cast<uint8_t*>(d_valid), static_cast<uint64_t*>(d_bitmap),
                        static_cast<hipStream_t>(stream));
}

int cmtv_register_keys(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, cmtv_keyset** out) {
  if (!out) return CMTV_EINVAL;
  *out = nullptr;
  // 512 KiB of comb per key; 2^20 keys would already be 512 GiB
  if (!ctx || n_keys == 0 || n_keys > (1u << 20) || !pk) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  return cmtv::register_keys_locked(ctx, n_keys, pk, out);
}

int cmtv_keyset_cache(cmtv_ctx* ctx, size_t max_sets) {
  if (!ctx || max_sets > 4096) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  (void)hipStreamSynchronize(ctx->stream);
  while (ctx->keysets.size() > max_sets) {
    cmtv_keyset_free(ctx->keysets.front().second);
    ctx->keysets.erase(ctx->keysets.begin());
  }
  ctx->keyset_cap = max_sets;
  return CMTV_OK;
}

}  // extern "C"

namespace cmtv {

int register_keys_locked(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, cmtv_keyset** out) {
  int rc = ensure_bcomb(ctx);
  if (rc != CMTV_OK) return rc;
  auto* ks = new (std::nothrow) cmtv_keyset();
  if (!ks) return CMTV_ENOMEM;
  ks->ctx = ctx;
  ks->n = n_keys;
  ks->pk.assign(pk, pk + 32 * n_keys);
  DevBuf scratch;
  hipError_t e = hipMalloc(&ks->d_pk, 32 * n_keys);
  if (e == hipSuccess) e = hipMalloc(&ks->d_ok, n_keys);
  if (e == hipSuccess) e = hipMalloc(&ks->d_tab, n_keys * (size_t)kCombWords * sizeof(uint32_t));
  if (e == hipSuccess)
    e = scratch.ensure((size_t)std::min<size_t>(n_keys, kCombKeyChunk) * kCombScratchWordsPerKey * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemcpyAsync(ks->d_pk, pk, 32 * n_keys, hipMemcpyHostToDevice, ctx->stream);
  for (size_t c = 0; e == hipSuccess && c < n_keys; c += kCombKeyChunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(kCombKeyChunk, n_keys - c);
    e = launch_comb_build(cn, ks->d_pk + 8 * c, ks->d_ok + c, ks->d_tab + c * (size_t)kCombWords,
                          static_cast<uint32_t*>(scratch.p), true, ctx->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  scratch.release();
  if (e != hipSuccess) {
    cmtv_keyset_free(ks);
    return hip_fail(e);
  }
  *out = ks;
  return CMTV_OK;
}

const cmtv_keyset* keyset_for_locked(cmtv_ctx* ctx, const uint8_t* pk32, size_t n_keys) {
  if (!ctx->keyset_cap || n_keys == 0) return nullptr;
  std::string key(reinterpret_cast<const char*>(pk32), 32 * n_keys);
  for (auto& e : ctx->keysets)
    if (e.first == key) return e.second;
  cmtv_keyset* ks = nullptr;
  if (register_keys_locked(ctx, n_keys, pk32, &ks) != CMTV_OK) return nullptr;  // generic path instead
  if (ctx->keysets.size() >= ctx->keyset_cap) {
    cmtv_keyset_free(ctx->keysets.front().second);
    ctx->keysets.erase(ctx->keysets.begin());
  }
  ctx->keysets.emplace_back(std::move(key), ks);
  return ks;
}

bool keyset_cache_enabled(const cmtv_ctx* ctx) { return ctx->keyset_cap != 0; }

}  // namespace cmtv

extern "C" {

void cmtv_keyset_free(cmtv_keyset* ks) {
  if (!ks) return;
  (void)hipSetDevice(ks->ctx->device);
  if (ks->d_pk) (void)hipFree(ks->d_pk);
  if (ks->d_ok) (void)hipFree(ks->d_ok);
  if (ks->d_tab) (void)hipFree(ks->d_tab);
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
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  const size_t msg_bytes = msg_off[n];
  // staging layout: [key_idx n*4][sig n*64][off (n+1)*4][msg msg_bytes + 16]
  const size_t o_idx = 0, o_sig = align_up(4 * n, 256), o_off = align_up(o_sig + 64 * n, 256);
  const size_t o_msg = align_up(o_off + 4 * (n + 1), 256), in_bytes = align_up(o_msg + msg_bytes + 16, 256);
  const size_t words = (n + 63) / 64;
  const size_t o_bm = 0, o_valid = align_up(8 * words, 256), out_bytes = align_up(o_valid + n, 256);
  hipError_t e;
  if ((e = ctx->h_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->h_out.ensure(out_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_out.ensure(out_bytes)) != hipSuccess) return hip_fail(e);
  auto* hin = static_cast<uint8_t*>(ctx->h_in.p);
  std::memcpy(hin + o_idx, key_idx, 4 * n);
  std::memcpy(hin + o_sig, sig, 64 * n);
  std::memcpy(hin + o_off, msg_off, 4 * (n + 1));
  if (msg_bytes) std::memcpy(hin + o_msg, msg, msg_bytes);
  std::memset(hin + o_msg + msg_bytes, 0, 16);
  auto* din = static_cast<uint8_t*>(ctx->d_in.p);
  auto* dout = static_cast<uint8_t*>(ctx->d_out.p);
  if ((e = hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess) return hip_fail(e);
  int rc = enqueue_verify_keyed(ctx, ks, n, reinterpret_cast<uint32_t*>(din + o_idx), din + o_sig, din + o_msg,
                                reinterpret_cast<uint32_t*>(din + o_off), mode, dout + o_valid,
                                reinterpret_cast<uint64_t*>(dout + o_bm), ctx->stream);
  if (rc != CMTV_OK) return rc;
  auto* hout = static_cast<uint8_t*>(ctx->h_out.p);
  if ((e = hipMemcpyAsync(hout, dout, out_bytes, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess) return hip_fail(e);
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e);
  harvest_timing(ctx);
  uint64_t invalid = 0;
  const uint8_t* hv = hout + o_valid;
  for (size_t i = 0; i < n; i++) invalid += hv[i] == 0;
  ctx->stats.invalid += invalid;
  if (out_valid) std::memcpy(out_valid, hv, n);
  if (out_bitmap) std::memcpy(out_bitmap, hout + o_bm, 8 * words);
  return CMTV_OK;
}

int cmtv_verify_ed25519_indexed_device(cmtv_ctx* ctx, const cmtv_keyset* ks, size_t n, const void* d_key_idx,
                                       const void* d_sig, const void* d_msg, const void* d_msg_off, uint32_t mode,
                                       void* d_valid, void* d_bitmap, void* stream) {
  if (!ctx || !ks || ks->ctx != ctx || mode > CMTV_MODE_ZIP215 || n > (1ull << 31)) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  if (!d_key_idx || !d_sig || !d_msg || !d_msg_off || (!d_valid && !d_bitmap)) return CMTV_EINVAL;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  return enqueue_verify_keyed(ctx, ks, n, static_cast<const uint32_t*>(d_key_idx),
                              static_cast<const uint8_t*>(d_sig), static_cast<const uint8_t*>(d_msg),
                              static_cast<const uint32_t*>(d_msg_off), mode, static_cast<uint8_t*>(d_valid),
                              static_cast<uint64_t*>(d_bitmap), static_cast<hipStream_t>(stream));
}

int cmtv_pubkeys_ed25519(cmtv_ctx* ctx, size_t n, const uint8_t* seeds, uint8_t* out_pk) {
  if (!ctx || n > (1ull << 31) || (n && (!seeds || !out_pk))) return CMTV_EINVAL;
  if (n == 0) return CMTV_OK;
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  hipError_t e;
  if ((e = ctx->d_in.ensure(32 * n)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_out.ensure(32 * n)) != hipSuccess) return hip_fail(e);
  if ((e = hipMemcpyAsync(ctx->d_in.p, seeds, 32 * n, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
    return hip_fail(e);
  for (size_t c = 0; c < n; c += kChunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(kChunk, n - c);
    if ((e = launch_pubkey(cn, static_cast<uint8_t*>(ctx->d_in.p) + 32 * c, ctx->d_btab,
                           static_cast<uint8_t*>(ctx->d_out.p) + 32 * c, ctx->stream)) != hipSuccess)
      return hip_fail(e);
  }
  if ((e = hipMemcpyAsync(out_pk, ctx->d_out.p, 32 * n, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess)
    return hip_fail(e);
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e);
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
  std::lock_guard<std::mutex> g(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CMTV_ENODEV;
  const size_t msg_bytes = msg_off[n];
  const size_t o_seed = 0, o_idx = align_up(32 * nseeds, 256), o_off = align_up(o_idx + (key_idx ? 4 * n : 0), 256);
  const size_t o_msg = align_up(o_off + 4 * (n + 1), 256), in_bytes = align_up(o_msg + msg_bytes + 16, 256);
  hipError_t e;
  if ((e = ctx->h_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_in.ensure(in_bytes)) != hipSuccess) return hip_fail(e);
  if ((e = ctx->d_out.ensure(64 * n)) != hipSuccess) return hip_fail(e);
  auto* hin = static_cast<uint8_t*>(ctx->h_in.p);
  std::memcpy(hin + o_seed, seeds, 32 * nseeds);
  if (key_idx) std::memcpy(hin + o_idx, key_idx, 4 * n);
  std::memcpy(hin + o_off, msg_off, 4 * (n + 1));
  if (msg_bytes) std::memcpy(hin + o_msg, msg, msg_bytes);
  auto* din = static_cast<uint8_t*>(ctx->d_in.p);
  if ((e = hipMemcpyAsync(din, hin, in_bytes, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess) return hip_fail(e);
  for (size_t c = 0; c < n; c += kChunk) {
    const uint32_t cn = (uint32_t)std::min<size_t>(kChunk, n - c);
    if ((e = launch_sign(cn, key_idx ? din + o_seed : din + o_seed + 32 * c, key_idx ? din + o_idx + 4 * c : nullptr,
                         din + o_msg,
                         din + o_off + 4 * c, ctx->d_btab, static_cast<uint8_t*>(ctx->d_out.p) + 64 * c,
                         ctx->stream)) != hipSuccess)
      return hip_fail(e);
  }
  if ((e = hipMemcpyAsync(out_sig, ctx->d_out.p, 64 * n, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess)
    return hip_fail(e);
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(e);
  return CMTV_OK;
}

}  // extern "C"
