// runtime_internal.h -- functions shared between runtime.cpp and the host-side
// commit / batch layers (commit.cpp). Not part of the C ABI.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <mutex>

struct cmtv_ctx;
struct cmtv_keyset;

namespace cmtv {

// Locks the context and makes its device current on this thread.
int ctx_lock(cmtv_ctx* ctx, std::unique_lock<std::mutex>& lk);
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
// cache). Caller holds the context lock.
int verify_templated_locked(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint32_t* msg_off,
                            const void* tmpls, size_t n_tmpls, const uint8_t* blob, size_t blob_len,
                            const uint32_t* tidx, const uint8_t* commit_flag, const int64_t* sec,
                            const int32_t* nanos, uint32_t mode, uint8_t* out_valid,
                            const cmtv_keyset* ks = nullptr, const uint32_t* key_idx = nullptr);

// cmtv_keyset_cache: the registered key set of these n 32-byte keys (built on
// first use), or NULL when the cache is off or registration failed.
const cmtv_keyset* keyset_for_locked(cmtv_ctx* ctx, const uint8_t* pk32, size_t n_keys);
bool keyset_cache_enabled(const cmtv_ctx* ctx);

// Host-side phase clock (CMTV_HOST_PHASES=1, read at open): where a call's
// host time goes, summed over the context's life and printed as one JSON line
// on stderr by cmtv_close. phase_now is 0 when the clock is off.
enum HostPhase { kPhPrepare, kPhStage, kPhLaunch, kPhWait, kPhPost, kPhReplay, kPhCount };
uint64_t phase_now(const cmtv_ctx* ctx);
void phase_add(cmtv_ctx* ctx, int phase, uint64_t t0);
int register_keys_locked(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, cmtv_keyset** out, uint32_t flags);

}  // namespace cmtv
