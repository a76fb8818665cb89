// runtime_internal.h -- functions shared between runtime.cpp and the host-side
// commit / batch layers (commit.cpp). Not part of the C ABI.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <functional>
#include <mutex>
#include <vector>

struct cmtv_ctx;
struct cmtv_keyset;

namespace cmtv {

// Locks the context and makes its device current on this thread.
int ctx_lock(cmtv_ctx* ctx, std::unique_lock<std::mutex>& lk);
// Re-takes a released context lock (the pipeline, between chunks) after any
// thread waiting in ctx_lock got it first.
void bulk_relock(cmtv_ctx* ctx, std::unique_lock<std::mutex>& lk);
uint32_t ctx_default_mode(const cmtv_ctx* ctx);
// Internal pseudo-mode selecting the sr25519 kernel in verify_host_locked /
// enqueue paths (the ABI's mode argument is Ed25519-only).
constexpr uint32_t kModeSr25519 = 0x100;

// Whether cmtv_verdict_cache is on (commit.cpp then prefetches light calls).
bool cache_enabled(const cmtv_ctx* ctx);

// Host buffers in, verdicts out (through the verdict cache when enabled);
// caller holds the context lock.
int verify_host_locked(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                       const uint32_t* msg_off, uint32_t mode, uint8_t* out_valid, uint64_t* out_bitmap);

// Commit signatures whose sign-bytes are written on the device from per-commit
// templates (signbytes.h): tmpls is an array of n_tmpls SbTemplate over
// `blob`; msg_off must hold the message offsets from sb_msg_len. With ks the
// keys are registered (key_idx into ks, no pk). Verdicts only (no verdict
// cache). tidx null: every signature uses template 0; key_idx null (with
// ks): signature i is by key i. Caller holds the context lock.
int verify_templated_locked(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint32_t* msg_off,
                            const void* tmpls, size_t n_tmpls, const uint8_t* blob, size_t blob_len,
                            const uint32_t* tidx, const uint8_t* commit_flag, const int64_t* sec,
                            const int32_t* nanos, uint32_t mode, uint8_t* out_valid,
                            const cmtv_keyset* ks = nullptr, const uint32_t* key_idx = nullptr,
                            uint32_t msg_bound = 0, const std::function<bool()>* between = nullptr,
                            bool* between_ok = nullptr);
// (msg_off null: no message offsets, every message at most msg_bound bytes;
// derived from the templates here unless the fused small-batch path, which
// never reads them, runs the batch; between: run once the kernels are
// enqueued, before the wait -- its answer in *between_ok)

// A single commit's n contiguous 64-byte signatures -- and, for the generic
// kernels (pk set: the validator set's n packed 32-byte keys), its keys --
// copied toward device memory before the commit is planned (the copy
// overlaps the plan); the templated batch that follows picks them up (no-op
// unless one live device, n <= the zero-copy size and CMTV_EARLY_SIGS is on;
// with pk, only past the row kernels' band, which keep reading their
// staging in place). Caller holds the lock.
int stage_sigs_early_locked(cmtv_ctx* ctx, const uint8_t* sigs, size_t n, const uint8_t* pk = nullptr);
// Forgets early-staged signatures (ctx_lock does it on every new lock hold;
// cmtv_verify_commit also on every exit). Caller holds the lock.
void clear_early_locked(cmtv_ctx* ctx);

// cmtv_keyset_cache: the registered key set of these n 32-byte keys (built on
// first use), or NULL when the cache is off or registration failed.
const cmtv_keyset* keyset_for_locked(cmtv_ctx* ctx, const uint8_t* pk32, size_t n_keys);
// The set keyset_for_locked last returned for this very key array (pointer
// and count; no byte compared), or NULL; and whether a set holds exactly
// these keys (the byte compare).
const cmtv_keyset* keyset_guess_locked(const cmtv_ctx* ctx, const uint8_t* pk32, size_t n_keys);
bool keyset_holds_locked(const cmtv_keyset* ks, const uint8_t* pk32, size_t n_keys);
// The speculative VerifyCommit's threshold in signatures (commit.cpp
// verify_commit_spec): CMTV_SPEC_MIN (default 2,048), 0 with CMTV_SPEC=0.
uint32_t spec_min(const cmtv_ctx* ctx);
bool keyset_cache_enabled(const cmtv_ctx* ctx);

// Host-side phase clock (CMTV_HOST_PHASES=1, read at open): where a call's
// host time goes, summed over the context's life and printed as one JSON line
// on stderr by cmtv_close. phase_now is 0 when the clock is off.
// The pipeline's phases (pipeline.cpp): per-commit plan, pinned-staging
// pack, submission (under the context lock), waits for chunk verdicts and
// replay; each summed over the host worker threads' wall time, not CPU time;
// pipe_cut: the submitting thread's serial chunk cut (its plan windows apart).
enum HostPhase {
  kPhPrepare, kPhStage, kPhLaunch, kPhWait, kPhPost, kPhReplay,
  kPhPipePlan, kPhPipePack, kPhPipeSubmit, kPhPipeWait, kPhPipeReplay, kPhKeyset, kPhEarly, kPhPipeCut, kPhCount
};
uint64_t phase_now(const cmtv_ctx* ctx);
void phase_add(cmtv_ctx* ctx, int phase, uint64_t t0);
int register_keys_locked(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, cmtv_keyset** out, uint32_t flags);
// phase_add with a duration measured elsewhere (pipeline; lock held)
void phase_add_ns(cmtv_ctx* ctx, int phase, uint64_t ns);

// ---------------------------------------------------------------- bulk lanes
// Large cross-height batches (pipeline.cpp) run through a per-device bulk
// lane: its own H2D (copy) and kernel (exec, lowest priority) streams, its
// own lane-kernel scratch and kBulkSlots pinned / device staging slots, so a
// chunk neither queues behind nor shares buffers with other calls, and the
// context lock is held only while a chunk is enqueued.
//
// One chunk's staging, in one pinned block copied to the device at once:
//   key  u32 validator index (registered keys) or 32-byte key, per signature
//   sig  64 bytes, off u32 message offsets (m + 1), tidx u32 commit template,
//   flag u8 (1 = BlockIDFlagCommit), sec i64, nanos i32 per signature,
//   tmpls SbTemplate per commit, blob the templates' bytes;
// on the device k_sign_bytes then writes the sign-bytes after it (o_msg).
//
// A DIRECT chunk (the caller's flags, timestamps and signatures in
// cmtv_alloc_pinned memory, every commit's plan a prefix of its signatures,
// registered keys) packs nothing per signature: the pinned staging holds only
//   tmpls, blob, desc (one BulkDesc per commit, signbytes.h)
// and the device gets the caller's arrays by DMA -- up to kBulkSpansMax spans
// of its pinned memory, copied to o_arena -- from which k_bulk_gather builds
// the per-signature arrays above (device-only, after in_bytes).
constexpr int kBulkSlotsMax = 4;
constexpr int kBulkSpansMax = 4;
struct BulkSpan {
  const uint8_t* host = nullptr;  // pinned source, 256-byte aligned
  size_t bytes = 0;
  size_t dev_off = 0;  // from o_arena, 256-byte aligned (host and device agree mod 256)
};
struct BulkLayout {
  size_t m = 0, n_tmpls = 0, blob_len = 0;
  uint64_t msg_bytes = 0;  // direct: an upper bound (the device computes the offsets)
  bool keyed = false, direct = false;
  bool masked = false;  // submitted to the lane's CU-masked exec stream
  size_t o_key = 0, o_sig = 0, o_off = 0, o_tidx = 0, o_flag = 0, o_sec = 0, o_nanos = 0, o_tmpl = 0, o_blob = 0;
  size_t o_desc = 0, o_cbase = 0, o_arena = 0, arena_bytes = 0;
  int n_spans = 0;
  BulkSpan spans[kBulkSpansMax];
  size_t in_bytes = 0, o_msg = 0, dev_bytes = 0;
  void compute();
};
// The caller's pinned blocks (cmtv_alloc_pinned), sorted by address: a
// snapshot for one pipeline call (context lock held)
struct PinnedRange {
  uintptr_t base;
  size_t bytes;
};
void pinned_ranges_locked(cmtv_ctx* ctx, std::vector<PinnedRange>& out);
// [p, p + bytes) lies in one of the caller's pinned blocks (lock held)
bool pinned_holds_locked(const cmtv_ctx* ctx, const void* p, size_t bytes);
std::mutex& bulk_mutex(cmtv_ctx* ctx);
class HostPool;
// the context's worker pool (created on first use; bulk lock held)
HostPool& host_pool(cmtv_ctx* ctx);
struct PipeConfig {
  size_t min_sigs, chunk;
  int slots;
  bool enabled;
  bool direct = true;  // CMTV_PIPE_DIRECT=0: always pack (A/B, tests)
  size_t chunk_masked = 0;  // a chunk on a CU-masked lane (latency_recent): one round of its CUs
  // a direct chunk ends where its DMA extents pass span_factor x the bytes
  // its plans read + span_slack (pipeline.cpp cut_chunk; tests shrink them)
  uint64_t span_factor = 4, span_slack = 64ull << 20;
  // bulk_prepare outside the context lock (CMTV_SPLIT_SUBMIT)
  bool split_submit = true;
};
PipeConfig pipe_config(const cmtv_ctx* ctx);
// Latency calls beside the pipeline (runtime.cpp cmtv_ctx::lat_window_ns):
// note_latency marks one (a single commit, a small batch); latency_recent is
// true within the window after one -- the pipeline then submits its chunks
// to the CU-masked exec stream (BulkLayout::masked). BulkBusy marks a
// pipeline call in flight (its scope).
void note_latency(cmtv_ctx* ctx);
// CMTV_CALL_TRACE (diagnostics, runtime.cpp cmtv_ctx::call_trace)
bool call_trace_on(const cmtv_ctx* ctx);
uint64_t call_trace_now();
void call_trace_begin_locked(cmtv_ctx* ctx);
void call_trace_record_locked(cmtv_ctx* ctx, uint64_t t_entry, uint64_t t_locked);
bool latency_recent(const cmtv_ctx* ctx);
struct BulkBusy {
  explicit BulkBusy(cmtv_ctx* c);
  ~BulkBusy();
  cmtv_ctx* ctx;
};
// A latency call's scope (context lock held): while a pipeline call is in
// flight and the latency window is open, each live device's normal stream
// is swapped for its bulk lane's latency stream -- the CUs the masked bulk
// chunks leave free -- and swapped back, ordered after it, on exit.
struct LatencyStreams {
  explicit LatencyStreams(cmtv_ctx* c);
  ~LatencyStreams();
  LatencyStreams(const LatencyStreams&) = delete;
  LatencyStreams& operator=(const LatencyStreams&) = delete;
  cmtv_ctx* ctx;
  uint64_t swapped = 0;  // device indices
};
// live device indices, in shard order (context lock held)
void live_devices_locked(cmtv_ctx* ctx, std::vector<size_t>& out);
// the pinned staging of (dev, slot), grown to L.in_bytes (bulk lock held)
int bulk_stage(cmtv_ctx* ctx, size_t dev, int slot, const BulkLayout& L, uint8_t** host);
// enqueues the lane-only part of the chunk staged in (dev, slot): H2D, the
// direct chunk's DMAs and gather, the sign-bytes (bulk lock held, not the
// context lock)
int bulk_prepare(cmtv_ctx* ctx, size_t dev, int slot, const BulkLayout& L, const cmtv_keyset* ks);
// ... then its verification (ks: by registered key) and verdict bitmap D2H
// (context lock held)
int bulk_submit_locked(cmtv_ctx* ctx, size_t dev, int slot, const BulkLayout& L, const cmtv_keyset* ks,
                       uint32_t mode);
// waits for the chunk in (dev, slot); *bitmap = its verdict words (pinned)
int bulk_wait(cmtv_ctx* ctx, size_t dev, int slot, const uint64_t** bitmap);
// after an error: waits for every bulk lane, clears sticky errors
void bulk_drain(cmtv_ctx* ctx);
// retires device dev after its HIP error (context lock held); false if it was
// the last live device
bool retire_device_locked(cmtv_ctx* ctx, size_t dev);
// the pipeline's per-call arrays, owned by the context (pipeline.cpp; freed
// by cmtv_close through pipe_workspace_free); bulk lock held
struct PipeWorkspace;
PipeWorkspace*& pipe_workspace(cmtv_ctx* ctx);
void pipe_workspace_free(PipeWorkspace* w);
// the context's invalid-verdict counter (context lock held)
void count_invalid_locked(cmtv_ctx* ctx, uint64_t n);
// cmtv_stats.direct_chunks (context lock held)
void count_direct_locked(cmtv_ctx* ctx);
// registered key set pins (context lock held): a pinned cached set is not
// freed by eviction until unpinned
void keyset_pin_locked(const cmtv_keyset* ks);
void keyset_unpin_locked(cmtv_ctx* ctx, const cmtv_keyset* ks);

}  // namespace cmtv
