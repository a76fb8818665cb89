// pipeline.cpp -- cmtv_verify_commits for large cross-height batches
// (blocksync and light-client replay: blockchain/v0/reactor.go:349-400,
// light/client.go:613-689; BASELINE configs[2], 100k commits x 150).
//
// The one-batch path (commit.cpp) plans, stages and replays a call on one
// thread with the context lock held throughout, and stages the whole batch
// before the first kernel starts. Here a call is cut into chunks of about
// CMTV_PIPE_CHUNK planned signatures (commit-aligned, one registered key set
// per chunk) that flow through the per-device bulk lanes (runtime.cpp):
//
//   plan     every commit's preamble and plan (the signatures the reference
//            loop can reach: types/validator_set.go:685-707, 740-762,
//            793-823), its template and sign-bytes lengths -- host workers
//   pack     a chunk's keys / indices, signatures, timestamps, flags and
//            templates into its slot's pinned staging -- host workers
//   submit   H2D on the lane's copy stream, k_sign_bytes + the verify kernel
//            + the bitmap D2H on its exec stream -- context lock held
//   replay   each commit's reference loop over the chunk's verdict bits
//            (commit_internal.h job_replay) -- host workers
//
// Chunk c+1 is packed while the device verifies chunk c, and chunk c-k is
// replayed while it does: with S slots per device and G devices, G x S
// chunks are in flight. Chunks go round-robin over the live devices, each
// with its own lane; a device that fails with a HIP error is retired and the
// chunks not yet replayed are run again on the others. Verdicts, errors and
// early exits are exactly the one-batch path's (the same plan and replay
// code, the same kernels).
#include <emmintrin.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "commit_internal.h"
#include "host_pool.h"
#include "runtime_internal.h"
#include "signbytes.h"

namespace cmtv {

namespace {

uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// The caller's arrays a direct chunk reads (BulkLayout), by class: the
// signatures, ts_seconds, ts_nanos and flags of its commits' plans. Each
// class's [lo, hi) over the chunk's commits; the DMA copies their union
// (classes closer than kSpanGap merged into one span).
constexpr int kClsSig = 0, kClsSec = 1, kClsNanos = 2, kClsFlags = 3, kClasses = 4;
constexpr uintptr_t kSpanGap = 64 * 1024;
struct SpanAcc {
  uintptr_t lo[kClasses], hi[kClasses];
  uint64_t need = 0;  // bytes the plans read
  SpanAcc() {
    for (int k = 0; k < kClasses; k++) {
      lo[k] = UINTPTR_MAX;
      hi[k] = 0;
    }
  }
  static void ranges(const cmtv_commit* cm, size_t m, uintptr_t* a, size_t* len) {
    a[kClsSig] = reinterpret_cast<uintptr_t>(cm->sigs + cm->sig_off[0]);
    len[kClsSig] = 64 * m;
    a[kClsSec] = reinterpret_cast<uintptr_t>(cm->ts_seconds);
    len[kClsSec] = 8 * m;
    a[kClsNanos] = reinterpret_cast<uintptr_t>(cm->ts_nanos);
    len[kClsNanos] = 4 * m;
    a[kClsFlags] = reinterpret_cast<uintptr_t>(cm->flags);
    len[kClsFlags] = m;
  }
  void add(const cmtv_commit* cm, size_t m) {
    uintptr_t a[kClasses];
    size_t len[kClasses];
    ranges(cm, m, a, len);
    for (int k = 0; k < kClasses; k++) {
      lo[k] = std::min(lo[k], a[k]);
      hi[k] = std::max(hi[k], a[k] + len[k]);
    }
    need += 77 * m;
  }
  // the same from the class starts ranges() gave (lengths: 64, 8, 4, 1 per signature)
  void add(const uintptr_t* a, size_t m) {
    static constexpr size_t w[kClasses] = {64, 8, 4, 1};
    for (int k = 0; k < kClasses; k++) {
      lo[k] = std::min(lo[k], a[k]);
      hi[k] = std::max(hi[k], a[k] + w[k] * m);
    }
    need += 77 * m;
  }
  // the merged spans (sorted by address): count, and [slo, shi) of each
  int merge(uintptr_t* slo, uintptr_t* shi, int* cls_span) const {
    int order[kClasses] = {0, 1, 2, 3};
    std::sort(order, order + kClasses, [&](int x, int y) { return lo[x] < lo[y]; });
    int ns = 0;
    for (int j = 0; j < kClasses; j++) {
      const int k = order[j];
      if (lo[k] >= hi[k]) {  // nothing of this class (m == 0 everywhere)
        cls_span[k] = -1;
        continue;
      }
      if (ns && lo[k] <= shi[ns - 1] + kSpanGap) {
        shi[ns - 1] = std::max(shi[ns - 1], hi[k]);
      } else {
        slo[ns] = lo[k];
        shi[ns] = hi[k];
        ns++;
      }
      cls_span[k] = ns - 1;
    }
    return ns;
  }
  // the classes' extents summed (>= merged_bytes when they do not overlap)
  uint64_t sum_bytes() const {
    uint64_t b = 0;
    for (int k = 0; k < kClasses; k++) b += lo[k] < hi[k] ? hi[k] - lo[k] : 0;
    return b;
  }
  uint64_t merged_bytes() const {
    uintptr_t slo[kClasses], shi[kClasses];
    int cs[kClasses];
    const int ns = merge(slo, shi, cs);
    uint64_t b = 0;
    for (int j = 0; j < ns; j++) b += shi[j] - slo[j];
    return b;
  }
};

struct Chunk {
  size_t c0 = 0, c1 = 0;              // commits [c0, c1)
  const cmtv_valset* vs = nullptr;    // the key class of its signatures
  const cmtv_keyset* ks = nullptr;    // registered keys, or null (generic kernel)
  size_t dev = 0;                     // where it was submitted
  int slot = 0;
  bool direct = false;                // DMA'd from the caller's pinned block (BulkLayout)
  SpanAcc acc;                        // direct: the classes' extents ...
  uintptr_t cls_lo[kClasses] = {};    // ... and where each class starts, host
  uint64_t cls_dev[kClasses] = {};    // and device (from o_arena)
  BulkLayout L;
};

// The first invalid verdict among batch bits [i0, i0 + m) as a plan index
// (m: all valid).
size_t first_invalid(const uint64_t* bm, size_t i0, size_t m) {
  const size_t end = i0 + m;
  for (size_t i = i0; i < end;) {
    const size_t b = i & 63, lim = std::min<size_t>(64 - b, end - i);
    uint64_t x = ~bm[i >> 6] >> b;
    if (lim < 64) x &= (1ull << lim) - 1;
    if (x) return i + (size_t)__builtin_ctzll(x) - i0;
    i += lim;
  }
  return m;
}

// The pinned block holding [p, p + len), or -1.
long find_block(const std::vector<PinnedRange>& pins, const void* p, size_t len) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = std::upper_bound(pins.begin(), pins.end(), a,
                             [](uintptr_t x, const PinnedRange& r) { return x < r.base; });
  if (it == pins.begin()) return -1;
  --it;
  if (a + len < a || a + len > it->base + it->bytes) return -1;
  return (long)(it - pins.begin());
}

// Copy into the pinned staging with non-temporal stores: the staging is
// written once by the host and read once by the H2D copy, so its lines need
// not be read for ownership or kept in the cache (the pack is bound by host
// memory traffic: ~165 B per signature instead of ~250). The writer calls
// nt_fence before its block's bytes may be read.
inline void nt_copy(uint8_t* dst, const uint8_t* src, size_t n) {
  const size_t head = std::min(n, (size_t)((16 - ((uintptr_t)dst & 15)) & 15));
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  for (; n >= 64; n -= 64, dst += 64, src += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + 48), d);
  }
  for (; n >= 16; n -= 16, dst += 16, src += 16)
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst), _mm_loadu_si128(reinterpret_cast<const __m128i*>(src)));
  std::memcpy(dst, src, n);
}

inline void nt_fence() { _mm_sfence(); }

// Two validator-set structs over the same arrays (a caller typically hands
// one struct per commit, all pointing at its set's arrays): one evaluation
// of the set serves both within a call.
inline bool same_arrays(const cmtv_valset* a, const cmtv_valset* b) {
  return a == b || (a->n_vals == b->n_vals && a->pubkeys == b->pubkeys && a->pk_off == b->pk_off &&
                    a->voting_power == b->voting_power);
}

// keys of vals are all 32 bytes and packed (what a registered key set needs)
bool packed_keys(const cmtv_valset* v) {
  if (!v->n_vals) return false;
  for (uint32_t i = 0; i <= v->n_vals; i++)
    if (v->pk_off[i] != 32 * i) return false;
  return true;
}

}  // namespace

// The pipeline's per-call arrays, kept by the context between calls
// (runtime_internal.h pipe_workspace).
struct PipeWorkspace {
  std::unique_ptr<uint32_t[]> pidx, pval;  // plan: commit / validator index per signature
  size_t cap_idx = 0, cap_val = 0;
  std::vector<uint64_t> base, mbytes, sp, mp, tp;
  std::vector<uint32_t> plen, tlen;
  // each commit's preamble outcome, kept from the plan to the replay
  std::vector<int32_t> early;
  std::vector<int64_t> needed;
  std::vector<const AddrIndex*> addr;  // LightTrusting
  // direct commits: their prefix plan's tally and the pinned block of their
  // arrays (direct[c] = 1)
  std::vector<uint8_t> direct;
  std::vector<int64_t> ptally;
  std::vector<uint32_t> pblock;
  // ... and where each of their array classes starts (SpanAcc::ranges, kept
  // by the parallel plan so the serial cut reads one sequential array)
  std::vector<std::array<uintptr_t, kClasses>> dspan;
  bool grow(size_t n, bool with_val) {
    if (cap_idx < n) {
      pidx.reset(new (std::nothrow) uint32_t[n]);
      cap_idx = pidx ? n : 0;
      if (!pidx) return false;
    }
    if (with_val && cap_val < n) {
      pval.reset(new (std::nothrow) uint32_t[n]);
      cap_val = pval ? n : 0;
      if (!pval) return false;
    }
    return true;
  }
};

void pipe_workspace_free(PipeWorkspace* w) { delete w; }

// The staging layout of one chunk (runtime_internal.h BulkLayout): the
// pipeline writes it, the bulk lane copies and launches on it.
void BulkLayout::compute() {
  auto up = [](size_t x) { return (x + 255) / 256 * 256; };
  if (direct) {
    // host part: templates, their bytes, descriptors; the rest device-only
    o_tmpl = 0;
    o_blob = up(n_tmpls * sizeof(SbTemplate));
    o_desc = up(o_blob + blob_len + 16);
    in_bytes = up(o_desc + n_tmpls * sizeof(BulkDesc));
    o_key = in_bytes;
    o_sig = up(o_key + 4 * m);
    o_off = up(o_sig + 64 * m);
    o_tidx = up(o_off + 4 * (m + 1));
    o_flag = up(o_tidx + 4 * m);
    o_sec = up(o_flag + m);
    o_nanos = up(o_sec + 8 * m);
    o_cbase = up(o_nanos + 4 * m);  // ctot, then cbase: n_tmpls words each
    o_arena = up(o_cbase + 8 * n_tmpls);
    o_msg = up(o_arena + arena_bytes);
    dev_bytes = up(o_msg + msg_bytes + 16);
    return;
  }
  o_key = 0;
  o_sig = up(keyed ? 4 * m : 32 * m);
  o_off = up(o_sig + 64 * m);
  o_tidx = up(o_off + 4 * (m + 1));
  o_flag = up(o_tidx + 4 * m);
  o_sec = up(o_flag + m);
  o_nanos = up(o_sec + 8 * m);
  o_tmpl = up(o_nanos + 4 * m);
  o_blob = up(o_tmpl + n_tmpls * sizeof(SbTemplate));
  in_bytes = up(o_blob + blob_len + 16);
  o_msg = in_bytes;  // device only: k_sign_bytes writes the messages here
  dev_bytes = up(o_msg + msg_bytes + 16);
}

bool pipeline_wanted(const cmtv_ctx* ctx, uint64_t n_sigs) {
  const PipeConfig pc = pipe_config(ctx);
  if (!pc.enabled || n_sigs < pc.min_sigs || cache_enabled(ctx)) return false;
  const char* v = std::getenv("CMTV_HOST_SIGNBYTES");  // host-encoded sign-bytes: one-batch path only
  return !(v && v[0] == '1');
}

namespace {

// The context lock re-taken for one step of the pipeline (bulk_relock: a
// waiting latency call goes first), released at scope end.
struct Relock {
  std::unique_lock<std::mutex>& lk;
  Relock(cmtv_ctx* c, std::unique_lock<std::mutex>& l) : lk(l) { bulk_relock(c, lk); }
  ~Relock() { lk.unlock(); }
  Relock(const Relock&) = delete;
  Relock& operator=(const Relock&) = delete;
};

// The pipeline proper; `pinned` collects the registered key sets it pins
// (released by the caller, also after an exception). Bulk lock held.
int run_pipeline(cmtv_ctx* ctx, const CommitsArgs& args, int* rcs, std::vector<const cmtv_keyset*>& pinned) {
  const size_t n = args.n;
  const uint32_t mode = args.mode;
  HostPool& pool = host_pool(ctx);
  const PipeConfig pc = pipe_config(ctx);
  const bool trusting = args.kind == CMTV_VERIFY_COMMIT_LIGHT_TRUSTING;
  uint64_t ph_plan = 0, ph_pack = 0, ph_submit = 0, ph_wait = 0, ph_replay = 0, ph_cut = 0;
  // ---- plan: each commit's preamble and plan, its template and sign-bytes
  // lengths -- window by window, just ahead of the chunk being cut, so the
  // planning of later commits overlaps the device's work on earlier chunks
  // per-call arrays live in the context's workspace: reused across calls,
  // so a pass over 15M signatures does not fault in 100+ MB of fresh pages
  PipeWorkspace*& wsp = pipe_workspace(ctx);
  if (!wsp) wsp = new (std::nothrow) PipeWorkspace();
  if (!wsp) return CMTV_ENOMEM;
  PipeWorkspace& W = *wsp;
  std::vector<uint64_t>& base = W.base;
  base.resize(n + 1);
  base[0] = 0;
  for (size_t c = 0; c < n; c++) base[c + 1] = base[c] + args.commits[c].n_sigs;
  if (!W.grow(base[n] + 1, trusting)) return CMTV_ENOMEM;
  uint32_t* const pidx_p = W.pidx.get();
  uint32_t* const pval_p = trusting ? W.pval.get() : nullptr;
  std::vector<uint32_t>& plen = W.plen;
  std::vector<uint32_t>& tlen = W.tlen;
  std::vector<uint64_t>& mbytes = W.mbytes;
  plen.resize(n);
  tlen.resize(n);
  mbytes.resize(n);
  W.early.resize(n);
  W.needed.resize(n);
  W.direct.resize(n);
  W.ptally.resize(n);
  W.pblock.resize(n);
  W.dspan.resize(n);
  // direct chunks (BulkLayout): on when the caller's arguments can be in
  // pinned blocks of this context and the registered-key cache is on
  std::vector<PinnedRange> pins;
  bool direct_on = false;
  static std::atomic<uint64_t> calls{0};
  const uint64_t call_id = ++calls;
  // LightTrusting: one address index per distinct (address array, size)
  std::map<std::pair<const uint8_t*, uint32_t>, AddrIndex> addr_index;
  if (trusting) {
    W.addr.resize(n);
    const AddrIndex* last = nullptr;
    std::pair<const uint8_t*, uint32_t> last_key{nullptr, 0};
    for (size_t c = 0; c < n; c++) {
      const cmtv_valset& v = args.vals[c];
      const auto key = std::make_pair(v.addrs, v.n_vals);
      if (!last || key != last_key) {
        auto it = addr_index.find(key);
        if (it == addr_index.end()) {
          it = addr_index.emplace(key, AddrIndex()).first;
          it->second.build(v.addrs, v.n_vals);
        }
        last = &it->second;
        last_key = key;
      }
      W.addr[c] = last;
    }
  }
  // a commit's job, its preamble's outcome restored after the plan
  auto job = [&](size_t c) {
    CommitJob J = args.job(c);
    if (trusting) J.addr = W.addr[c];
    return J;
  };
  // chunk-local offsets of each commit's first signature / sign-byte / template byte
  std::vector<uint64_t>& sp = W.sp;
  std::vector<uint64_t>& mp = W.mp;
  std::vector<uint64_t>& tp = W.tp;
  sp.resize(n);
  mp.resize(n);
  tp.resize(n);
  // the exact sign-bytes of a planned commit (pidx: its plan)
  auto exact_mbytes = [](const CommitJob& J, const uint32_t* pi, size_t m, const TplLens& tlz) {
    const cmtv_commit* cm = J.commit;
    const uint8_t* fl = cm->flags;
    const int64_t* se = cm->ts_seconds;
    const int32_t* na = cm->ts_nanos;
    uint64_t mb = 0;
    if (pi[m - 1] - pi[0] == m - 1) {  // a contiguous plan (the common case)
      const uint32_t a = pi[0];
      for (size_t k = 0; k < m; k++) mb += msg_len(tlz, fl[a + k] == kFlagCommit, se[a + k], na[a + k]);
    } else {
      for (size_t k = 0; k < m; k++) {
        const uint32_t idx = pi[k];
        mb += msg_len(tlz, fl[idx] == kFlagCommit, se[idx], na[idx]);
      }
    }
    return mb;
  };
  // A direct commit (BulkLayout): its plan is its signatures [0, m) --
  // VerifyCommit: every flag Commit or Nil; VerifyCommitLight: Commit flags
  // up to the +2/3 threshold -- from a set of packed 32-byte keys, 64-byte
  // signatures back to back, and its four arrays aligned and inside ONE of the
  // caller's pinned blocks. Nothing per signature is then packed on the host:
  // the plan costs one pass over the flags (and powers) and the signature
  // offsets. Sets plen, tlen, mbytes (an upper bound: every message at its
  // template's longest) and the direct fields; false: the general plan.
  auto plan_direct = [&](size_t c, const CommitJob& J) -> bool {
    const cmtv_commit* cm = J.commit;
    const cmtv_valset* v = J.vals;
    const uint32_t n_s = cm->n_sigs;
    if (n_s != v->n_vals) return false;
    // per distinct set of this call (the id keeps a set freed and
    // reallocated at the same address between calls from hitting): whether
    // its keys are packed, its total power, and -- VerifyCommitLight -- the
    // prefix an all-Commit commit of it reaches (the plan then depends on the
    // set alone)
    struct SetInfo {
      const cmtv_valset* v = nullptr;
      uint64_t call = 0;
      bool packed = false;
      int64_t total = 0;
      uint32_t light_m = 0;
      int64_t light_tally = 0;
    };
    thread_local SetInfo si;
    if (!si.v || si.call != call_id || !same_arrays(v, si.v)) {
      si.v = v;
      si.call = call_id;
      si.packed = packed_keys(v);
      si.total = 0;
      for (uint32_t i = 0; i < v->n_vals; i++) si.total += v->voting_power[i];
      int64_t t = 0;
      uint32_t m = 0;
      for (uint32_t i = 0; i < v->n_vals; i++) {
        t += v->voting_power[i];
        m = i + 1;
        if (t > J.needed) break;
      }
      si.light_m = m;
      si.light_tally = t;
    }
    if (!si.packed) return false;
    const uint8_t* fl = cm->flags;
    // every flag of [0, k) is BlockIDFlagCommit (eight at a time)
    auto all_commit = [fl](uint32_t k) {
      uint64_t bad = 0;
      uint32_t i = 0;
      for (; i + 8 <= k; i += 8) {
        uint64_t w;
        std::memcpy(&w, fl + i, 8);
        bad |= w ^ 0x0202020202020202ull;
      }
      for (; i < k; i++) bad |= fl[i] ^ kFlagCommit;
      return bad == 0;
    };
    int64_t tally = 0;
    uint32_t m = 0;
    if (J.kind == CMTV_VERIFY_COMMIT) {
      m = n_s;
      if (all_commit(n_s)) {
        tally = si.total;
      } else {
        const int64_t* vp = v->voting_power;
        uint32_t bad = 0;
        for (uint32_t i = 0; i < n_s; i++) {  // branch-free: the compiler vectorises it
          const uint8_t f = fl[i];
          const bool fb = f == kFlagCommit;
          bad |= (uint32_t)(!fb & (f != kFlagNil));
          tally += fb ? vp[i] : 0;
        }
        if (bad) return false;
      }
    } else {
      // J.needed is the set's (total * 2 / 3, as when si was filled)
      m = si.light_m;
      tally = si.light_tally;
      if (!all_commit(m)) return false;
    }
    uint32_t blk = UINT32_MAX;
    if (m) {
      const uint32_t* so = cm->sig_off;
      const uint32_t s0 = so[0];
      if ((uint64_t)s0 + 64ull * m > UINT32_MAX) return false;
      uint32_t bad = 0;
      for (uint32_t i = 1; i <= m; i++) bad |= so[i] ^ (s0 + 64u * i);  // vectorised
      if (bad) return false;
      uintptr_t* a = W.dspan[c].data();
      size_t len[kClasses];
      SpanAcc::ranges(cm, m, a, len);
      if ((a[kClsSig] & 7) || (a[kClsSec] & 7) || (a[kClsNanos] & 3)) return false;
      thread_local long hint = -1;
      for (int k = 0; k < kClasses; k++) {
        const PinnedRange* h = hint >= 0 && (size_t)hint < pins.size() ? &pins[(size_t)hint] : nullptr;
        long b;
        if (h && a[k] >= h->base && a[k] + len[k] >= a[k] && a[k] + len[k] <= h->base + h->bytes)
          b = hint;
        else
          b = hint = find_block(pins, reinterpret_cast<const void*>(a[k]), len[k]);
        if (b < 0 || (blk != UINT32_MAX && (uint32_t)b != blk)) return false;
        blk = (uint32_t)b;
      }
      TplLens tl;
      tlen[c] = (uint32_t)commit_template_lens(J.chain_id_len, cm, &tl.pre_commit, &tl.pre_nil, &tl.post);
      mbytes[c] = (uint64_t)m * msg_len_bound(tl);
    }
    plen[c] = m;
    W.direct[c] = 1;
    W.ptally[c] = tally;
    W.pblock[c] = blk;
    return true;
  };
  size_t planned_upto = 0;
  auto plan_window = [&](uint64_t want_sigs) {
    const uint64_t t0 = now_ns();
    size_t b = planned_upto;
    while (b < n && base[b] - base[planned_upto] < want_sigs) b++;
    if (b == planned_upto) b++;
    const size_t a = planned_upto;
    pool.parallel_for(b - a, 64, [&](size_t lo, size_t hi) {
      thread_local Seen seen;
      // each distinct validator set's total power once (job_preamble)
      const cmtv_valset* tot_vs = nullptr;
      int64_t tot = 0;
      for (size_t c = a + lo; c < a + hi; c++) {
        CommitJob J = job(c);
        if (!tot_vs || !same_arrays(J.vals, tot_vs)) {
          tot_vs = J.vals;
          tot = 0;
          for (uint32_t i = 0; i < tot_vs->n_vals; i++) tot += tot_vs->voting_power[i];
        }
        J.has_total = true;
        J.total = tot;
        job_preamble(J);
        W.early[c] = J.early;
        W.needed[c] = J.needed;
        W.direct[c] = 0;
        plen[c] = tlen[c] = 0;
        mbytes[c] = 0;
        if (J.early != 1) continue;
        if (direct_on && plan_direct(c, J)) continue;
        uint32_t* pi = pidx_p + base[c];
        const size_t m = job_plan(J, pi, trusting ? pval_p + base[c] : nullptr, seen);
        plen[c] = (uint32_t)m;
        if (!m) continue;
        TplLens tl;
        tlen[c] = (uint32_t)commit_template_lens(J.chain_id_len, J.commit, &tl.pre_commit, &tl.pre_nil, &tl.post);
        mbytes[c] = exact_mbytes(J, pi, m, tl);
      }
    });
    planned_upto = b;
    ph_plan += now_ns() - t0;
  };

  std::unique_lock<std::mutex> lk;
  int rc = ctx_lock(ctx, lk);
  if (rc != CMTV_OK) return rc;
  const bool keyed_mode = keyset_cache_enabled(ctx);
  std::vector<size_t> live;
  live_devices_locked(ctx, live);
  pinned_ranges_locked(ctx, pins);
  direct_on = pc.direct && keyed_mode && !trusting && !pins.empty();
  lk.unlock();

  // ---- chunks, cut on the fly: commit-aligned, about `per` planned
  // signatures each (at least the kernels' full-rate size, pc.chunk, and at
  // least two per device when the call is large enough to split), one key
  // class per chunk when the keyset cache can serve it
  std::vector<Chunk> chunks;
  uint64_t per = 0;
  bool ramp = false;
  size_t cursor = 0;  // next commit to put in a chunk
  const cmtv_valset* last_vs = nullptr;
  bool last_packed = false;
  const uint64_t max_mb = max_batch_msg_bytes();
  auto cut_chunk = [&]() -> int {  // appends the next chunk; CMTV_OK or an error
    struct CutClock {  // ph_cut: this cut's time, its plan windows apart
      uint64_t &cut, &plan, t0, plan0;
      ~CutClock() { cut += (now_ns() - t0) - (plan - plan0); }
    } cut_clock{ph_cut, ph_plan, now_ns(), ph_plan};
    if (per == 0) {
      // the first window sets the chunk size from its plan ratio
      plan_window(std::max<uint64_t>(pc.chunk, 1));
      const uint64_t ws = base[planned_upto], wp = [&] {
        uint64_t x = 0;
        for (size_t c = 0; c < planned_upto; c++) x += plen[c];
        return x;
      }();
      const uint64_t est = ws ? (uint64_t)((double)base[n] * ((double)wp / (double)ws)) : 0;
      uint64_t nc = std::max<uint64_t>(1, est / pc.chunk);
      const uint64_t spread = std::min<uint64_t>(2 * live.size(), est / std::max<size_t>(pc.min_sigs, 1));
      nc = std::max(nc, spread);
      per = std::max<uint64_t>(1, (est + nc - 1) / nc);
      const bool long_call = est / pc.chunk >= 4;
      // a long call runs chunks of pc.chunk planned signatures at most (the
      // default, 2^20, is one full round of the batched registered-key lane
      // kernel: 2,048 waves of 64 lanes x 8 signatures; a chunk just past it
      // would start a second, nearly empty round), and ramps up: its first
      // chunks are 1/16, 1/4 and 1/2 of that, so the device starts after a
      // fraction of a chunk's pack instead of a whole one
      if (long_call) {
        ramp = true;
        per = pc.chunk;
      }
    }
    uint64_t want = per;
    // the ramp: 1/16, 1/4, 1/2 of a chunk (2^16 signatures take the one-
    // signature-per-lane keyed kernel at two waves per SIMD, 2^18 and 2^19
    // the KB = 4 batch); measured on MI355X (tools/ramp_ab.sh, 100k x 150,
    // two alternating rounds): 40.9-41.1 ms per pass against 41.3-41.6 with
    // 1/8, 1/4, 1/2 and 42.3 without a ramp
    static constexpr int ramp_sh[] = {4, 2, 1};
    if (ramp && chunks.size() < 3) want = std::max<uint64_t>(per >> ramp_sh[chunks.size()], 1);
    Chunk ch;
    ch.c0 = cursor;
    // near a latency call the chunk runs on the CU-masked lane: no more than
    // one round of the CUs it keeps
    ch.L.masked = latency_recent(ctx);
    if (ch.L.masked) want = std::min<uint64_t>(want, pc.chunk_masked);
    bool cls_set = false;
    // direct class: the pinned block of a direct chunk's commits, -1 for a
    // packed chunk (a chunk is one or the other)
    bool dcls_set = false;
    long dcls = -1;
    uint64_t s = 0, mb = 0, tb = 0;
    size_t c = cursor;
    // the commits of the chunk; with per_commit_cap a direct chunk also ends
    // where its DMA extents outgrow its plans (below). The common case runs
    // without it and checks the extents once, for the whole chunk, from the
    // plan's per-commit class starts (W.dspan); only a chunk that fails that
    // check is cut again commit by commit (round 6: the per-commit extents
    // were ~40% of the serial cut, tests/host/pipebench's pipe_cut phase)
    auto scan = [&](bool per_commit_cap) {
      cls_set = dcls_set = false;
      dcls = -1;
      ch.vs = nullptr;
      ch.acc = SpanAcc();
      s = mb = tb = 0;
      c = cursor;
      for (; c < n; c++) {
        // plan a chunk's worth at a time: each window is one parallel_for (a
        // wake-up of every worker), so windows of 64k signatures cost ~230
        // wake-ups per 15M-signature call
        if (c == planned_upto)
          plan_window(std::max<uint64_t>(want - std::min(want, s), std::max<uint64_t>(pc.chunk, 65536)));
        const bool dir = plen[c] && W.direct[c];
        if (plen[c]) {
          const long dc = dir ? (long)W.pblock[c] : -1;
          if (dcls_set && dc != dcls) break;
          if (!dcls_set) {
            dcls = dc;
            dcls_set = true;
          }
        }
        if (plen[c] && keyed_mode) {
          const cmtv_valset* v = &args.vals[c];
          if (!last_vs || !same_arrays(v, last_vs)) {
            last_vs = v;
            last_packed = packed_keys(v);
          }
          const cmtv_valset* cls = last_packed ? v : nullptr;
          if (cls_set && !((cls == nullptr) == (ch.vs == nullptr) &&
                           (!cls || same_arrays(ch.vs, cls) || same_keys(ch.vs, cls))))
            break;
          if (!cls_set) {
            ch.vs = cls;
            cls_set = true;
          }
        }
        // cut below the target (a commit that would cross it opens the next
        // chunk), unless the chunk would be empty
        if (s && s + plen[c] > want) break;
        // ... and below the one-batch path's sign-bytes span per launch (its
        // message offsets are 32-bit): a commit that would cross it opens the
        // next chunk
        if (s && mb + mbytes[c] >= max_mb) break;
        sp[c] = s;
        mp[c] = mb;
        tp[c] = tb;
        s += plen[c];
        mb += mbytes[c];
        tb += tlen[c];
        if (s >= want) {
          if (dir && per_commit_cap) ch.acc.add(W.dspan[c].data(), plen[c]);
          c++;
          break;
        }
        if (dir && per_commit_cap) {
          // a direct chunk's DMA covers its classes' extents: it ends at a
          // commit past which it would copy far more than its plans read (a
          // caller's arrays scattered over its pinned block)
          ch.acc.add(W.dspan[c].data(), plen[c]);
          const uint64_t cap = pc.span_factor * ch.acc.need + pc.span_slack;
          if (ch.acc.sum_bytes() > cap && ch.acc.merged_bytes() > cap) {
            c++;
            break;
          }
        }
      }
    };
    scan(false);
    if (dcls_set && dcls >= 0) {
      // a direct chunk (every planned commit of it direct): its extents
      for (size_t k = cursor; k < c; k++)
        if (plen[k]) ch.acc.add(W.dspan[k].data(), plen[k]);
      const uint64_t cap = pc.span_factor * ch.acc.need + pc.span_slack;
      if (ch.acc.sum_bytes() > cap && ch.acc.merged_bytes() > cap) scan(true);
    }
    ch.c1 = c;
    cursor = c;
    ch.L.m = s;
    ch.L.n_tmpls = ch.c1 - ch.c0;
    ch.L.blob_len = tb;
    ch.L.msg_bytes = mb;
    if (mb >= max_mb) return CMTV_EINVAL;  // one commit's sign-bytes alone reach the span
    if (keyed_mode && ch.vs && ch.L.m) {
      Relock g(ctx, lk);
      ch.ks = keyset_for_locked(ctx, ch.vs->pubkeys, ch.vs->n_vals);
      if (ch.ks && std::find(pinned.begin(), pinned.end(), ch.ks) == pinned.end()) {
        keyset_pin_locked(ch.ks);
        pinned.push_back(ch.ks);
      }
    }
    ch.L.keyed = ch.ks != nullptr;
    ch.direct = dcls_set && dcls >= 0 && ch.L.m;
    if (ch.direct && !ch.ks) {
      // no registered key set (registration failed): pack this chunk after
      // all -- the same prefix plans, written out, with exact sign-bytes
      pool.parallel_for(ch.c1 - ch.c0, 64, [&](size_t lo, size_t hi) {
        thread_local Seen seen;
        for (size_t k = ch.c0 + lo; k < ch.c0 + hi; k++) {
          if (!W.direct[k]) continue;
          W.direct[k] = 0;
          if (!plen[k]) continue;
          CommitJob J = job(k);
          J.early = W.early[k];
          J.needed = W.needed[k];
          uint32_t* pi = pidx_p + base[k];
          (void)job_plan(J, pi, nullptr, seen);  // == the prefix [0, plen)
          SbTemplate tpl;
          put_commit_template(nullptr, 0, J.chain_id, J.chain_id_len, J.commit, &tpl);
          mbytes[k] = exact_mbytes(J, pi, plen[k], TplLens{tpl.pre_commit_len, tpl.pre_nil_len, tpl.post_len});
        }
      });
      uint64_t x = 0;
      for (size_t k = ch.c0; k < ch.c1; k++) {
        mp[k] = x;
        x += mbytes[k];
      }
      ch.L.msg_bytes = x;
      ch.direct = false;
    }
    if (ch.direct) {
      // the DMA spans: the classes' extents, merged, each landing at a
      // device offset congruent to its host address mod 256 (so the
      // caller's 8-byte alignment holds on the device)
      uintptr_t slo[kClasses], shi[kClasses];
      int cs[kClasses];
      const int ns = ch.acc.merge(slo, shi, cs);
      size_t at = 0;
      for (int j = 0; j < ns; j++) {
        at = (at + 255) / 256 * 256 + (slo[j] & 255);
        ch.L.spans[j] = BulkSpan{reinterpret_cast<const uint8_t*>(slo[j]), (size_t)(shi[j] - slo[j]), at};
        at += shi[j] - slo[j];
      }
      ch.L.n_spans = ns;
      ch.L.arena_bytes = at;
      for (int k = 0; k < kClasses; k++) {
        ch.cls_lo[k] = ch.acc.lo[k];
        ch.cls_dev[k] = cs[k] < 0 ? 0 : ch.L.spans[cs[k]].dev_off + (ch.acc.lo[k] - slo[cs[k]]);
      }
      ch.L.direct = true;
    }
    ch.L.compute();
    chunks.push_back(ch);
    return CMTV_OK;
  };

  // ---- the chunk loop
  // a direct chunk's host part: each commit's template and descriptor
  auto pack_direct = [&](Chunk& ch, uint8_t* h) {
    const BulkLayout& L = ch.L;
    auto* tmpls = reinterpret_cast<SbTemplate*>(h + L.o_tmpl);
    uint8_t* blob = h + L.o_blob;
    auto* desc = reinterpret_cast<BulkDesc*>(h + L.o_desc);
    pool.parallel_for(ch.c1 - ch.c0, 64, [&](size_t b, size_t e) {
      for (size_t c = ch.c0 + b; c < ch.c0 + e; c++) {
        const size_t tl = c - ch.c0;
        const uint32_t m = plen[c];
        if (!m) {
          tmpls[tl] = SbTemplate{};
          desc[tl] = BulkDesc{};
          continue;
        }
        const cmtv_commit* cm = &args.commits[c];
        put_commit_template(blob, tp[c], args.chain_id, args.chain_id_len, cm, &tmpls[tl]);
        uintptr_t a[kClasses];
        size_t len[kClasses];
        SpanAcc::ranges(cm, m, a, len);
        BulkDesc d;
        d.sig = ch.cls_dev[kClsSig] + (a[kClsSig] - ch.cls_lo[kClsSig]);
        d.sec = ch.cls_dev[kClsSec] + (a[kClsSec] - ch.cls_lo[kClsSec]);
        d.nanos = ch.cls_dev[kClsNanos] + (a[kClsNanos] - ch.cls_lo[kClsNanos]);
        d.flags = ch.cls_dev[kClsFlags] + (a[kClsFlags] - ch.cls_lo[kClsFlags]);
        d.sp = (uint32_t)sp[c];
        d.m = m;
        desc[tl] = d;
      }
    });
  };
  auto pack = [&](Chunk& ch, uint8_t* h) {
    if (ch.direct) return pack_direct(ch, h);
    const BulkLayout& L = ch.L;
    auto* kidx = reinterpret_cast<uint32_t*>(h + L.o_key);
    uint8_t* pk = h + L.o_key;
    uint8_t* sg = h + L.o_sig;
    auto* off = reinterpret_cast<uint32_t*>(h + L.o_off);
    auto* tidx = reinterpret_cast<uint32_t*>(h + L.o_tidx);
    uint8_t* flag = h + L.o_flag;
    auto* sec = reinterpret_cast<int64_t*>(h + L.o_sec);
    auto* nanos = reinterpret_cast<int32_t*>(h + L.o_nanos);
    auto* tmpls = reinterpret_cast<SbTemplate*>(h + L.o_tmpl);
    uint8_t* blob = h + L.o_blob;
    pool.parallel_for(ch.c1 - ch.c0, 16, [&](size_t b, size_t e) {
      for (size_t c = ch.c0 + b; c < ch.c0 + e; c++) {
        const size_t m = plen[c];
        if (!m) continue;
        const cmtv_commit* cm = &args.commits[c];
        const cmtv_valset* vals = &args.vals[c];
        const uint32_t tl = (uint32_t)(c - ch.c0);
        SbTemplate t;
        put_commit_template(blob, tp[c], args.chain_id, args.chain_id_len, cm, &t);
        tmpls[tl] = t;
        const uint32_t* pi = pidx_p + base[c];
        const uint32_t* pv = trusting ? pval_p + base[c] : pi;
        const size_t i0 = sp[c];
        uint64_t mo = mp[c];
        const TplLens tlz{t.pre_commit_len, t.pre_nil_len, t.post_len};
        // the common case, column by column: a contiguous plan whose
        // validators are the commit's indices and whose signatures are all
        // 64 bytes, back to back
        const uint32_t a = pi[0];
        bool run = !trusting && pi[m - 1] - a == m - 1 && cm->sig_off[a + m] - cm->sig_off[a] == 64 * m;
        for (size_t k = 0; run && k < m; k++) run = cm->sig_off[a + k + 1] - cm->sig_off[a + k] == 64;
        if (run) {
          nt_copy(sg + 64 * i0, cm->sigs + cm->sig_off[a], 64 * m);
          nt_copy(reinterpret_cast<uint8_t*>(sec + i0), reinterpret_cast<const uint8_t*>(cm->ts_seconds + a), 8 * m);
          nt_copy(reinterpret_cast<uint8_t*>(nanos + i0), reinterpret_cast<const uint8_t*>(cm->ts_nanos + a), 4 * m);
          const uint8_t* fl = cm->flags + a;
          for (size_t k = 0; k < m; k++) flag[i0 + k] = fl[k] == kFlagCommit;
          for (size_t k = 0; k < m; k++) tidx[i0 + k] = tl;
          if (L.keyed) {
            for (size_t k = 0; k < m; k++) kidx[i0 + k] = a + (uint32_t)k;
          } else if (vals->pk_off[a + m] - vals->pk_off[a] == 32 * m) {
            std::memcpy(pk + 32 * i0, vals->pubkeys + vals->pk_off[a], 32 * m);  // planned keys are 32 bytes
          } else {
            for (size_t k = 0; k < m; k++) std::memcpy(pk + 32 * (i0 + k), vals->pubkeys + vals->pk_off[a + k], 32);
          }
          const int64_t* se = cm->ts_seconds + a;
          const int32_t* na = cm->ts_nanos + a;
          for (size_t k = 0; k < m; k++) {
            off[i0 + k] = (uint32_t)mo;
            mo += msg_len(tlz, fl[k] == kFlagCommit, se[k], na[k]);
          }
          continue;
        }
        for (size_t k = 0; k < m; k++) {
          const size_t i = i0 + k;
          const uint32_t idx = pi[k], vi = pv[k];
          if (L.keyed)
            kidx[i] = vi;
          else
            std::memcpy(pk + 32 * i, vals->pubkeys + vals->pk_off[vi], 32);
          const uint32_t s0 = cm->sig_off[idx];
          if (cm->sig_off[idx + 1] - s0 == 64)
            std::memcpy(sg + 64 * i, cm->sigs + s0, 64);
          else
            std::memset(sg + 64 * i, 0, 64);  // invalid whatever the device says (job_replay)
          const bool fb = cm->flags[idx] == kFlagCommit;
          const int64_t se = cm->ts_seconds[idx];
          const int32_t na = cm->ts_nanos[idx];
          flag[i] = fb ? 1 : 0;
          sec[i] = se;
          nanos[i] = na;
          tidx[i] = tl;
          off[i] = (uint32_t)mo;
          mo += msg_len(tlz, fb, se, na);
        }
      }
      nt_fence();  // this block's streaming stores are visible before the H2D reads them
    });
    off[L.m] = (uint32_t)L.msg_bytes;
  };
  auto replay = [&](Chunk& ch, const uint64_t* bm) {
    pool.parallel_for(ch.c1 - ch.c0, 32, [&](size_t b, size_t e) {
      thread_local Seen seen;
      for (size_t c = ch.c0 + b; c < ch.c0 + e; c++) {
        const size_t i0 = sp[c];
        CommitJob J = job(c);
        J.early = W.early[c];
        J.needed = W.needed[c];
        if (W.direct[c]) {  // a prefix plan: its first invalid bit decides
          const size_t m = plen[c];
          rcs[c] = replay_prefix(J, m, W.ptally[c], m ? first_invalid(bm, i0, m) : 0);
          continue;
        }
        rcs[c] = job_replay(J, pidx_p + base[c], plen[c],
                            [bm, i0](size_t j) {
                              const size_t i = i0 + j;
                              return ((bm[i >> 6] >> (i & 63)) & 1) != 0;
                            },
                            seen);
      }
    });
  };

  size_t next_retire = 0, retired = 0;
  long bad_dev = -1;
  for (;;) {
    const size_t G = live.size();
    const size_t S = (size_t)pc.slots;
    if (G == 0) {
      rc = CMTV_ENODEV;
      break;
    }
    rc = CMTV_OK;
    bad_dev = -1;
    std::deque<size_t> inflight;
    size_t rr = 0;
    auto retire = [&](size_t c) -> int {
      Chunk& ch = chunks[c];
      const uint64_t* bm = nullptr;
      if (ch.L.m) {
        const uint64_t tw = now_ns();
        const int r = bulk_wait(ctx, ch.dev, ch.slot, &bm);
        ph_wait += now_ns() - tw;
        if (r != CMTV_OK) {
          bad_dev = (long)ch.dev;
          return r;
        }
      }
      const uint64_t tr = now_ns();
      replay(ch, bm);
      if (ch.L.m) {
        uint64_t valid = 0;
        for (size_t w = 0; w < ch.L.m / 64; w++) valid += (uint64_t)__builtin_popcountll(bm[w]);
        if (ch.L.m & 63) valid += (uint64_t)__builtin_popcountll(bm[ch.L.m / 64] & ((1ull << (ch.L.m & 63)) - 1));
        Relock g(ctx, lk);
        count_invalid_locked(ctx, ch.L.m - valid);
      }
      ph_replay += now_ns() - tr;
      retired = c + 1;  // chunks retire in order
      return CMTV_OK;
    };
    for (size_t c = next_retire; rc == CMTV_OK; c++) {
      if (c == chunks.size()) {
        if (cursor == n) break;
        if ((rc = cut_chunk()) != CMTV_OK) break;
      }
      while (rc == CMTV_OK && inflight.size() >= G * S) {
        rc = retire(inflight.front());
        inflight.pop_front();
      }
      if (rc != CMTV_OK) break;
      Chunk& ch = chunks[c];
      if (ch.L.m == 0) {  // nothing to verify: replayed in order with the others
        inflight.push_back(c);
        continue;
      }
      ch.dev = live[rr % G];
      ch.slot = (int)((rr / G) % S);
      rr++;
      uint8_t* h = nullptr;
      const uint64_t tk = now_ns();
      rc = bulk_stage(ctx, ch.dev, ch.slot, ch.L, &h);
      if (rc != CMTV_OK) {
        bad_dev = (long)ch.dev;
        break;
      }
      pack(ch, h);
      const uint64_t ts = now_ns();
      ph_pack += ts - tk;
      // the lane-only part first, outside the context lock (a latency call
      // on the context never waits behind it), then the launch under it
      if (pc.split_submit) rc = bulk_prepare(ctx, ch.dev, ch.slot, ch.L, ch.ks);
      if (rc == CMTV_OK) {
        Relock g(ctx, lk);
        if (!pc.split_submit) rc = bulk_prepare(ctx, ch.dev, ch.slot, ch.L, ch.ks);
        if (rc == CMTV_OK) rc = bulk_submit_locked(ctx, ch.dev, ch.slot, ch.L, ch.ks, mode);
        if (rc == CMTV_OK && ch.direct) count_direct_locked(ctx);
      }
      ph_submit += now_ns() - ts;
      if (rc != CMTV_OK) {
        bad_dev = (long)ch.dev;
        break;
      }
      inflight.push_back(c);
    }
    while (rc == CMTV_OK && !inflight.empty()) {
      rc = retire(inflight.front());
      inflight.pop_front();
    }
    next_retire = retired;
    if (rc == CMTV_OK) break;
    // a failure: nothing of this attempt stays in flight; a device's own HIP
    // error retires it and the chunks not yet replayed run on the others
    bulk_drain(ctx);
    Relock g(ctx, lk);
    if (rc != CMTV_EHIP || bad_dev < 0 || !retire_device_locked(ctx, (size_t)bad_dev)) break;
    // chunks are replayed in submission (= chunk) order, so the replayed
    // ones are exactly [0, next_retire): the rest run again
    live_devices_locked(ctx, live);
  }
  {
    Relock g(ctx, lk);
    phase_add_ns(ctx, kPhPipePlan, ph_plan);
    phase_add_ns(ctx, kPhPipeCut, ph_cut);
    phase_add_ns(ctx, kPhPipePack, ph_pack);
    phase_add_ns(ctx, kPhPipeSubmit, ph_submit);
    phase_add_ns(ctx, kPhPipeWait, ph_wait);
    phase_add_ns(ctx, kPhPipeReplay, ph_replay);
  }
  return rc;
}

}  // namespace

int verify_commits_pipeline(cmtv_ctx* ctx, const CommitsArgs& args, int* rcs) {
  std::unique_lock<std::mutex> bulk(bulk_mutex(ctx));
  const BulkBusy busy(ctx);
  std::vector<const cmtv_keyset*> pinned;
  pinned.reserve(8);
  int rc;
  bool threw = false;
  // no C++ exception crosses the C ABI: a failed allocation (std::bad_alloc)
  // or thread creation (std::system_error) is the call's error code, after
  // everything the call enqueued has drained
  try {
    rc = run_pipeline(ctx, args, rcs, pinned);
  } catch (const std::bad_alloc&) {
    rc = CMTV_ENOMEM;
    threw = true;
  } catch (...) {
    rc = CMTV_EINVAL;
    threw = true;
  }
  if (threw) bulk_drain(ctx);
  if (!pinned.empty()) {
    std::unique_lock<std::mutex> lk;
    (void)ctx_lock(ctx, lk);
    for (auto* ks : pinned) keyset_unpin_locked(ctx, ks);
  }
  return rc;
}

}  // namespace cmtv
