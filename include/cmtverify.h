/*
 * cmtverify.h -- C ABI of libcmtverify.so, the MI355X (gfx950) batch Ed25519
 * verifier behind CometBFT's commit-verification path.
 *
 * Drop-in boundary. The reference (Tendermint/CometBFT v0.34.28, pure Go,
 * CGO_ENABLED=0 at /root/reference/Makefile:11) verifies one signature at a
 * time through the Go interface
 *     crypto.PubKey.VerifySignature(msg, sig []byte) bool
 *         /root/reference/crypto/crypto.go:25
 *         /root/reference/crypto/ed25519/ed25519.go:148-155
 * called from the tally loops of
 *     ValidatorSet.VerifyCommit            types/validator_set.go:667-714
 *     ValidatorSet.VerifyCommitLight       types/validator_set.go:722-765
 *     ValidatorSet.VerifyCommitLightTrusting types/validator_set.go:775-826
 * Every entry point below is what a cgo binding for that path binds (see
 * INTEGRATION.md for the Go side: crypto.BatchVerifier and the rewritten
 * VerifyCommit* bodies that replay the reference loop over the verdicts).
 *
 * Conventions
 *   - Return 0 on success, a negative CMTV_E* code otherwise; never abort, no
 *     exceptions cross the ABI. Verdicts are only meaningful on success.
 *   - Caller-owned host buffers are read during the call only; the library
 *     copies them into its own pinned staging and keeps no pointer after
 *     returning (cgo pointer rules).
 *   - Thread-safe: a context serialises its own calls with a mutex and calls
 *     hipSetDevice on entry (Go goroutines migrate between OS threads).
 *     Device-resident (_device) calls on different streams are ordered
 *     against each other wherever they share context scratch.
 *   - One context may drive several devices (cmtv_open_devices): host-buffer
 *     batches are split into contiguous 64-aligned shards, one per device,
 *     and the shards' verdict bitmaps are all-gathered over RCCL (xGMI) so
 *     the caller gets one verdict vector. A Go node is one process, so this
 *     is how it uses every GPU of the node.
 *   - Messages: one flat byte buffer + (n+1) uint32 offsets; message i is
 *     msg[msg_off[i] .. msg_off[i+1]).
 *   - Bitmaps: uint64 words, bit (i % 64) of word (i / 64) = verdict of i.
 *   - Modes: CMTV_MODE_GO_STDLIB reproduces Go 1.19 crypto/ed25519.Verify (the
 *     semantics this reference runs); CMTV_MODE_ZIP215 is the cofactored
 *     ZIP-215 rule of upstream curve25519-voi.
 */
#ifndef CMTVERIFY_H
#define CMTVERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMTV_ABI_VERSION 11

enum {
  CMTV_OK = 0,
  CMTV_EINVAL = -1,  /* bad argument (null pointer, n too large, bad mode) */
  CMTV_ENODEV = -2,  /* no usable gfx950 device                           */
  CMTV_ENOMEM = -3,  /* device or pinned host allocation failed           */
  CMTV_EHIP = -4,    /* HIP runtime error (launch, copy, sync)            */
  CMTV_ERCCL = -5,   /* collective failure (multi-device gather)          */
  CMTV_ECOMMIT = -6  /* commit verification failed: see the message out   */
};

enum { CMTV_MODE_GO_STDLIB = 0, CMTV_MODE_ZIP215 = 1 };

typedef struct cmtv_ctx cmtv_ctx;
typedef struct cmtv_batch cmtv_batch;
typedef struct cmtv_keyset cmtv_keyset;

typedef struct cmtv_config {
  int32_t device;        /* HIP device ordinal; -1 = current device          */
  uint32_t default_mode; /* mode used by cmtv_batch_* and cmtv_verify_commit */
  uint32_t flags;        /* reserved, must be 0                              */
  uint32_t reserved;
} cmtv_config;

typedef struct cmtv_stats {
  uint64_t calls;          /* verify calls                        */
  uint64_t signatures;     /* signatures verified                 */
  uint64_t invalid;        /* signatures rejected                 */
  uint64_t kernel_launches;
  double device_ms;        /* summed kernel time of the TIMED calls (HIP
                              events; CMTV_TIMING=N times one call in N per
                              device, default 16): mean kernel time =
                              device_ms / timed_calls                     */
  double last_kernel_ms;   /* the most recent timed verify call    */
  uint64_t cache_hits;     /* verdicts served by the verdict cache */
  uint64_t cache_entries;  /* verdicts currently cached           */
  uint64_t keyed_launches; /* launches of the registered-key kernels */
  uint64_t sharded_calls;  /* batches split over more than one device */
  uint64_t gathers;        /* bitmap all-gathers (RCCL or peer copy) */
  uint64_t faults_injected;/* launches failed by the CMTV_FAULT_AT knob */
  uint32_t n_devices;      /* devices driven by the context       */
  uint32_t rccl;           /* 1: gathers run over an RCCL communicator */
  uint64_t fused_sign_bytes; /* templated batches whose sign-bytes the verify
                              kernel's helper wave wrote (no k_sign_bytes) */
  uint64_t device_failures;  /* devices retired after a HIP error          */
  uint64_t reshards;         /* host batches re-planned over the remaining
                              devices after such a failure               */
  uint64_t late_k_waves;     /* keyed split-kernel quad waves that stopped
                              waiting for the hash helper and hashed their own
                              signatures (timing only, never a verdict)  */
  uint32_t live_devices;     /* devices still taking work                 */
  uint32_t reserved;
  uint64_t timed_calls;      /* calls whose kernel time device_ms holds   */
  uint64_t rccl_failures;    /* RCCL all-gathers that failed; that gather
                              and every later one of the context used peer
                              copies (rccl drops to 0) unless
                              CMTV_NO_RCCL_FALLBACK is set               */
  uint64_t polled_calls;     /* small host batches whose bitmap the host read
                              off the row kernel's completion flag, without
                              waiting for the kernel to retire
                              (CMTV_HOST_POLL)                           */
  uint64_t direct_chunks;    /* cross-height pipeline chunks DMA'd straight
                              from the caller's cmtv_alloc_pinned memory (no
                              host pack per signature)                   */
  uint64_t masked_chunks;    /* pipeline chunks run on the CU-masked exec
                              stream because a latency call (a single
                              commit) came within CMTV_LAT_WINDOW_MS      */
  uint64_t isolated_calls;   /* latency calls (a single commit, a small
                              cmtv_verify_commits) run on the CUs those
                              masked chunks leave free (CMTV_LAT_ISOLATE) */
} cmtv_stats;

/* One device's share of the context's work (cmtv_device_stats_get). */
typedef struct cmtv_device_stats {
  int32_t ordinal;          /* HIP ordinal                                 */
  uint32_t failed;          /* 1: retired after a HIP error                */
  uint64_t calls;           /* verify calls that ran on this device        */
  uint64_t signatures;
  uint64_t kernel_launches;
  double device_ms;         /* summed kernel time of this device's timed calls */
  uint64_t timed_calls;     /* ... and their number                        */
} cmtv_device_stats;

/* ------------------------------------------------------------ lifecycle */

/* Opens a context on one device: creates its stream, uploads the fixed-base
 * tables of (1..128)B, (1..128)[2^124]B and (1..128)[2^128]B (built on the
 * device), allocates pinned staging.
 * Replaces: nothing in the reference (it has no device state).
 * Environment (read at open): CMTV_ROW2_MAX / CMTV_ROW_MAX / CMTV_ROW_WAVES / CMTV_OCT_MAX /
 * CMTV_OCT_SPLIT_MAX / CMTV_QUAD_MAX / CMTV_QUAD_SPLIT_MAX / CMTV_KEYED_QUAD_MAX / CMTV_LANE_CHUNK
 * (kernel crossovers: Ed25519 batches up to CMTV_ROW2_MAX (256) take a whole
 * CU per signature (four waves; CMTV_ROW_WAVES=2: two), up to CMTV_ROW_MAX
 * (1536) one wave per signature, up to CMTV_OCT_MAX (2048) 8 lanes, up to
 * CMTV_QUAD_MAX (49152; sr25519 40000) 4 lanes, larger ones one lane), CMTV_FAULT_AT=N (test knob: the N-th verification
 * launch of the context fails with CMTV_EHIP without running; libs/fail
 * FAIL_TEST_INDEX analogue), CMTV_FORCE_WIDE=1 (test knob: the quad kernels
 * take the 64-window half-scalar fallback for every signature),
 * CMTV_FORCE_RCCL=1 (test knob: a one-rank RCCL communicator even over one
 * device, so a one-GPU box exercises the RCCL init and all-gather),
 * CMTV_FAULT_DEV=g (test knob: every launch on the context's g-th device
 * fails with a HIP error: host batches retire it and re-shard onto the other
 * devices), CMTV_FAULT_SYNC_DEV=g (test knob: device g's stream
 * synchronisation in a host batch reports a HIP error, i.e. a fault found
 * after the launch; same retirement), CMTV_FORCE_K_LATE=1 (test knob: the
 * keyed split kernel's quads never wait for the hash helper and hash their
 * signatures themselves), CMTV_RCCL_LIB=path (the RCCL library to dlopen
 * instead of the system librccl; with CMTV_FORCE_RCCL a repeated ordinal then
 * gets a multi-rank communicator: the one-GPU rehearsal of the RCCL path with
 * tests/host/librccl_stub.so), CMTV_ROW_FENCE=0 (test knob: no fence on the
 * row kernels' bitmap ring, see cmtv_verify_ed25519_device),
 * CMTV_NO_RCCL_FALLBACK=1 (a failed RCCL all-gather returns CMTV_ERCCL
 * instead of switching the context to peer copies), CMTV_QUAD_HS=0 (the
 * quad kernel's quads add both table entries of a window themselves:
 * k_verify_quad_split instead of k_verify_quad_hs), CMTV_HS_PRE=k (tuning:
 * the helper-summed kernel's helper adds the top k of [u]B's 16 comb
 * positions, default 6), CMTV_HOST_POLL=0 (a small single-device host batch
 * on a row kernel waits for its stream instead of polling the kernel's tagged
 * bitmap words: runtime.cpp wait_row_tags; the call may otherwise return
 * while the kernel's last waves retire, its verdicts already complete). */
int cmtv_open(const cmtv_config* cfg, cmtv_ctx** out);

/* Opens ONE context over several devices (a node is one
 * process; blockchain/v0/reactor.go:349-400 verifies from one goroutine).
 * devices[0..n_devices) are HIP ordinals; n_devices == 0 takes the list from
 * CMTVERIFY_DEVICES ("0,1,2,3" or "all"), or every visible gfx950 device when
 * it is unset. Each device gets its own stream, staging, fixed-base tables
 * and registered-key combs; when the ordinals are distinct an RCCL
 * communicator over them (ncclCommInitAll) carries the bitmap all-gather,
 * otherwise (a repeated ordinal, used to exercise sharding on one GPU) peer
 * copies do. A host-buffer batch is sharded over as many devices as get at
 * least CMTV_SHARD_MIN (default 8192) signatures each (a 40k batch takes 4
 * of 8 GPUs; below 2 x CMTV_SHARD_MIN it runs on one).
 * Device failure: a device whose launch, copy or sync fails with a HIP error
 * is retired (cmtv_stats.device_failures, cmtv_device_stats.failed), the RCCL
 * communicator is rebuilt over the others and the failed host batch is
 * re-planned over them and run again in the same call; later host batches
 * never use it. Device-resident calls that need a retired device return
 * CMTV_ENODEV (their inputs were on it).
 * Device-resident single-device calls (_device) run on devices[0].
 * cfg->device is ignored; cfg may be NULL (then CMTVERIFY_MODE = "go" |
 * "zip215" picks the default mode). */
int cmtv_open_devices(const cmtv_config* cfg, const int32_t* devices, size_t n_devices, cmtv_ctx** out);
int cmtv_device_count(const cmtv_ctx* ctx);
/* HIP ordinal / hipStream_t (as void*) of the context's g-th device */
int cmtv_device_ordinal(const cmtv_ctx* ctx, int g);
void* cmtv_device_stream(cmtv_ctx* ctx, int g);
/* Waits for every device stream of the context. */
int cmtv_sync(cmtv_ctx* ctx);
void cmtv_close(cmtv_ctx* ctx);
const char* cmtv_strerror(int code);
int cmtv_abi_version(void);
int cmtv_stats_get(cmtv_ctx* ctx, cmtv_stats* out);
/* Stats of the context's g-th device (0 <= g < cmtv_device_count). */
int cmtv_device_stats_get(cmtv_ctx* ctx, int g, cmtv_device_stats* out);
/* hipStream_t of the context (as void*), for callers that order their own
 * work with it (bench, multi-GPU gather). */
void* cmtv_stream(cmtv_ctx* ctx);

/* ------------------------------------------------------------ verification */

/* Batch verification from host buffers: n signatures, pk n x 32 bytes,
 * sig n x 64 bytes. out_valid: n bytes (0/1), out_bitmap (optional, may be
 * NULL): ceil(n/64) words. Each verdict equals
 *   PubKey(pk_i).VerifySignature(msg_i, sig_i)   crypto/ed25519/ed25519.go:148
 * for 32-byte keys and 64-byte signatures (callers handle other lengths, see
 * cmtv_batch_add). Blocking. */
int cmtv_verify_ed25519(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                        const uint32_t* msg_off, uint32_t mode, uint8_t* out_valid, uint64_t* out_bitmap);

/* Same, all buffers already resident in device memory (HBM); enqueued on
 * `stream` (a hipStream_t; NULL = the HIP null stream, as in every HIP API;
 * cmtv_stream() gives the context's own stream), non-blocking. d_valid
 * (n bytes) and d_bitmap (ceil(n/64) words) may each be NULL.
 * In-flight contract: any number of _device calls may be in flight on any
 * number of streams. Batches of the row kernels (n <= 1536 by default) pack
 * their bitmap through one slot of a 256-slot per-device ring; a slot whose
 * previous launch may still be running is fenced (the new launch's stream
 * waits for the old launch's event), so verdict words never depend on what
 * else is in flight. These calls record and wait on HIP events: do not
 * enqueue them inside a hipStreamBeginCapture region (graph replays would
 * reuse one ring slot without the fence). Returns CMTV_ENODEV once the
 * context's first device has been retired after a HIP error. */
int cmtv_verify_ed25519_device(cmtv_ctx* ctx, size_t n, const void* d_pk, const void* d_sig, const void* d_msg,
                               const void* d_msg_off, uint32_t mode, void* d_valid, void* d_bitmap, void* stream);

/* Multi-device, device-resident (bench / configs[2] replay): shard g has
 * n_shard[g] signatures whose inputs (layout as cmtv_verify_ed25519_device)
 * are resident on the context's g-th device. Every device verifies its shard
 * on its own stream; the shard bitmaps are then all-gathered (RCCL, in place)
 * so that each device's d_bitmap_all[g] -- G x W words, W = max over shards
 * of ceil(n_shard / 64), returned in *words_per_shard -- holds shard h's
 * verdict bits at words [h W, h W + ceil(n_shard[h] / 64)). d_valid[g]
 * (n_shard[g] bytes) may be NULL, or the array itself NULL. Non-blocking:
 * cmtv_sync waits. */
int cmtv_verify_ed25519_sharded_device(cmtv_ctx* ctx, const size_t* n_shard, const void* const* d_pk,
                                       const void* const* d_sig, const void* const* d_msg,
                                       const void* const* d_msg_off, uint32_t mode, void* const* d_valid,
                                       void* const* d_bitmap_all, size_t* words_per_shard);

/* Multi-device, device-resident, INDEPENDENT batches (one commit per device,
 * e.g. the configs[1] step at N GPUs): device g verifies its own n_dev[g]
 * signatures on its own stream and writes ceil(n_dev[g] / 64) verdict words
 * to d_bitmap[g] (and n_dev[g] bytes to d_valid[g] unless NULL). Nothing is
 * exchanged between devices: each batch's verdicts go to its own caller.
 * Non-blocking: cmtv_sync waits. */
int cmtv_verify_ed25519_multi_device(cmtv_ctx* ctx, const size_t* n_dev, const void* const* d_pk,
                                     const void* const* d_sig, const void* const* d_msg,
                                     const void* const* d_msg_off, uint32_t mode, void* const* d_valid,
                                     void* const* d_bitmap);

/* ------------------------------------------------------------ verdict cache */

/* Blocksync verifies each commit three times with the same (key, sign-bytes,
 * signature) triples: VerifyCommitLight in the reactor, then VerifyCommit
 * twice (blockchain/v0/reactor.go:366-400 -> state/validation.go:93,
 * state/execution.go:135). cmtv_verdict_cache(ctx, max_entries) keeps the
 * verdicts of the last max_entries verifications of the context (0 disables
 * and clears). Entries are matched on the full (mode, key, signature,
 * message) bytes, so a hit returns exactly the verdict the device would
 * compute. With the cache on, cmtv_verify_commit / cmtv_verify_commits also
 * verify a light call's remaining non-absent signatures in the same device
 * batch (their verdicts only fill the cache; the replay never reads them),
 * so the two full VerifyCommit calls that follow need no device work.
 * Applies to the host-buffer entry points (cmtv_verify_ed25519, batch,
 * commit). */
int cmtv_verdict_cache(cmtv_ctx* ctx, size_t max_entries);

/* A node verifies commit after commit against the same validator set.
 * cmtv_keyset_cache(ctx, max_sets) keeps the registered key sets
 * (cmtv_register_keys) of up to max_sets validator sets, built the first time
 * cmtv_verify_commit / cmtv_verify_commits see a set whose keys are all 32
 * bytes; later commits of that set are verified by key index (no
 * decompression of A, no doublings; same verdicts). Applies when the verdict
 * cache is off. 0 disables and frees the cached sets. 512 KiB of HBM per key. */
int cmtv_keyset_cache(cmtv_ctx* ctx, size_t max_sets);

/* ------------------------------------------------------------ sr25519 */

/* sr25519 (schnorrkel over ristretto255) batch verification, BASELINE
 * configs[4]. Each verdict equals
 *   sr25519.PubKey(pk_i).VerifySignature(msg_i, sig_i)   crypto/sr25519/pubkey.go:34-60
 * (go-schnorrkel v1.0.0: signing context "" + msg, ristretto255 decoding of the
 * key and of R, the schnorrkel marker bit sig[63] & 0x80, canonical s, merlin
 * challenge, R' = [s]B - [k]A compared with ristretto equality) for 32-byte
 * keys and 64-byte signatures; callers apply pubkey.go's length rules
 * (len(sig) != 64 -> false; the key is copied into a zeroed 32-byte array).
 * Buffers, ownership and blocking behaviour as cmtv_verify_ed25519. */
int cmtv_verify_sr25519(cmtv_ctx* ctx, size_t n, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                        const uint32_t* msg_off, uint8_t* out_valid, uint64_t* out_bitmap);

/* Same with device-resident inputs, enqueued on `stream` (as
 * cmtv_verify_ed25519_device). */
int cmtv_verify_sr25519_device(cmtv_ctx* ctx, size_t n, const void* d_pk, const void* d_sig, const void* d_msg,
                               const void* d_msg_off, void* d_valid, void* d_bitmap, void* stream);

/* ------------------------------------------------------------ registered keys */

/* A validator set signs commit after commit with the same keys (blocksync,
 * light-client and state-sync replay: blockchain/v0/reactor.go:366-400,
 * light/verifier.go:60-125, both ending in the VerifyCommit* loops above).
 * The reference decodes each key again inside every
 * PubKey.VerifySignature (crypto/ed25519/ed25519.go:154). cmtv_register_keys
 * decodes n_keys 32-byte keys once and builds, per key, the radix-256 comb
 * (e+1)*256^j*(-A) (j < 32, e < 128; 512 KiB of HBM per key), so that
 * indexed verification needs no decompression of A and no doublings.
 * Verdicts are identical to cmtv_verify_ed25519's on the same (pk, msg, sig):
 * a key that fails to decode makes every signature under it invalid, and the
 * key's original bytes are what SHA-512(R || A || M) hashes. Blocking. The
 * key set belongs to `ctx`: free it before cmtv_close(ctx). */
int cmtv_register_keys(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, cmtv_keyset** out);

/* cmtv_register_keys with flags. CMTV_KEYS_WIDE also builds each key's
 * radix-2^16 comb (e+1)*2^(16j)*(-A) (j < 16, e < 32768; 64 MiB of HBM per
 * key, n_keys <= 4096), which the one-signature-per-lane kernels of large
 * indexed batches then use: 32 table additions per signature instead of 64
 * (bulk replay of one validator set, BASELINE configs[2]). Same verdicts. */
enum { CMTV_KEYS_WIDE = 1 };
int cmtv_register_keys_ex(cmtv_ctx* ctx, size_t n_keys, const uint8_t* pk, uint32_t flags, cmtv_keyset** out);
void cmtv_keyset_free(cmtv_keyset* ks);
size_t cmtv_keyset_len(const cmtv_keyset* ks);

/* Verification of n signatures where signature i is by registered key
 * key_idx[i] (every index must be < cmtv_keyset_len: CMTV_EINVAL otherwise).
 * Buffers and outputs as in cmtv_verify_ed25519. Blocking. */
int cmtv_verify_ed25519_indexed(cmtv_ctx* ctx, const cmtv_keyset* ks, size_t n, const uint32_t* key_idx,
                                const uint8_t* sig, const uint8_t* msg, const uint32_t* msg_off, uint32_t mode,
                                uint8_t* out_valid, uint64_t* out_bitmap);

/* Same with device-resident inputs, enqueued on `stream` (NULL = HIP null
 * stream), non-blocking. An out-of-range d_key_idx entry gives an invalid
 * verdict (the kernel never reads outside the key set). */
int cmtv_verify_ed25519_indexed_device(cmtv_ctx* ctx, const cmtv_keyset* ks, size_t n, const void* d_key_idx,
                                       const void* d_sig, const void* d_msg, const void* d_msg_off, uint32_t mode,
                                       void* d_valid, void* d_bitmap, void* stream);

/* The same, sharded across the context's devices (see
 * cmtv_verify_ed25519_sharded_device for the layout): d_key_idx[g] indexes
 * the key set, which is registered on every device of the context. */
int cmtv_verify_ed25519_indexed_sharded_device(cmtv_ctx* ctx, const cmtv_keyset* ks, const size_t* n_shard,
                                               const void* const* d_key_idx, const void* const* d_sig,
                                               const void* const* d_msg, const void* const* d_msg_off,
                                               uint32_t mode, void* const* d_valid, void* const* d_bitmap_all,
                                               size_t* words_per_shard);

/* ------------------------------------------------------------ crypto.BatchVerifier mirror */

/* crypto.BatchVerifier as upstream CometBFT v0.38 defines it (not in this
 * v0.34 reference; the Go side is in INTEGRATION.md):
 *   Add(key PubKey, msg, sig []byte) error ;  Verify() (bool, []bool)
 * cmtv_batch_add never fails on malformed input: a signature whose length is
 * not 64 is recorded as invalid (ed25519.go:150); a key whose length is not 32
 * is recorded and reported as invalid with *deferred_panic set by
 * cmtv_batch_verify, so the Go replay can panic at the same index the
 * reference's sequential loop would (Go's ed25519.Verify panics on it). */
int cmtv_batch_new(cmtv_ctx* ctx, uint32_t mode, cmtv_batch** out);
int cmtv_batch_add(cmtv_batch* b, const uint8_t* pk, size_t pk_len, const uint8_t* msg, size_t msg_len,
                   const uint8_t* sig, size_t sig_len);
size_t cmtv_batch_len(const cmtv_batch* b);
/* out_valid: len bytes; *all_ok = 1 iff every entry is valid; bad_key_index:
 * first entry whose key length was not 32 (or -1). */
int cmtv_batch_verify(cmtv_batch* b, uint8_t* out_valid, int* all_ok, int64_t* bad_key_index);
void cmtv_batch_reset(cmtv_batch* b);
void cmtv_batch_free(cmtv_batch* b);

/* ------------------------------------------------------------ commit verification */

/* A commit and its validator set in struct-of-arrays form.
 *   types/block.go:575-600  Commit / CommitSig / BlockIDFlag (Absent=1, Commit=2, Nil=3)
 *   types/validator_set.go  ValidatorSet (Validators[i].PubKey, .VotingPower, .Address)
 * Sign-bytes are produced by the library's CanonicalVote encoder
 * (types/vote.go:93, types/canonical.go:56, canonical.pb.go:517). */
typedef struct cmtv_block_id {
  const uint8_t* hash;
  uint32_t hash_len;
  uint32_t psh_total;
  const uint8_t* psh_hash;
  uint32_t psh_hash_len;
} cmtv_block_id;

typedef struct cmtv_commit {
  int64_t height;
  int32_t round;
  cmtv_block_id block_id;
  uint32_t n_sigs;
  const uint8_t* flags;          /* n_sigs BlockIDFlag bytes              */
  const int64_t* ts_seconds;     /* n_sigs Unix seconds of CommitSig.Timestamp */
  const int32_t* ts_nanos;       /* n_sigs nanoseconds                    */
  const uint8_t* sigs;           /* concatenated signatures               */
  const uint32_t* sig_off;       /* n_sigs+1 offsets into sigs            */
  const uint8_t* val_addrs;      /* n_sigs x 20 (ValidatorAddress); may be NULL unless LightTrusting */
} cmtv_commit;

typedef struct cmtv_valset {
  uint32_t n_vals;
  const uint8_t* pubkeys;        /* concatenated public keys              */
  const uint32_t* pk_off;        /* n_vals+1 offsets into pubkeys         */
  const int64_t* voting_power;   /* n_vals                                */
  const uint8_t* addrs;          /* n_vals x 20; required for LightTrusting */
  const int64_t* proposer_priority; /* n_vals, optional (only printed in the
                                       double-vote error, Validator.String()) */
} cmtv_valset;

enum { CMTV_VERIFY_COMMIT = 0, CMTV_VERIFY_COMMIT_LIGHT = 1, CMTV_VERIFY_COMMIT_LIGHT_TRUSTING = 2 };

enum {
  CMTV_COMMIT_OK = 0,
  CMTV_COMMIT_ERR_SET_SIZE = 1,        /* ErrInvalidCommitSignatures        */
  CMTV_COMMIT_ERR_HEIGHT = 2,          /* ErrInvalidCommitHeight            */
  CMTV_COMMIT_ERR_BLOCK_ID = 3,        /* "invalid commit -- wrong block ID" */
  CMTV_COMMIT_ERR_WRONG_SIGNATURE = 4, /* "wrong signature (#%d): %X"       */
  CMTV_COMMIT_ERR_NOT_ENOUGH_POWER = 5,/* ErrNotEnoughVotingPowerSigned     */
  CMTV_COMMIT_ERR_DOUBLE_VOTE = 6,     /* "double vote from %v (%d and %d)" */
  CMTV_COMMIT_ERR_TRUST_LEVEL = 7,     /* zero denominator / int64 overflow */
  CMTV_COMMIT_PANIC_BAD_PUBKEY = 8,    /* the reference panics here (Go ed25519.Verify) */
  CMTV_COMMIT_PANIC_UNKNOWN_FLAG = 9   /* the reference panics here (CommitSig.BlockID) */
};

typedef struct cmtv_commit_result {
  int32_t code;        /* CMTV_COMMIT_*                                      */
  int32_t sig_index;   /* index the error refers to, or -1 (DOUBLE_VOTE: the
                          second commit index)                               */
  int64_t got;         /* ErrNotEnoughVotingPowerSigned.Got; DOUBLE_VOTE: the
                          first commit index                                 */
  int64_t needed;      /* ErrNotEnoughVotingPowerSigned.Needed; DOUBLE_VOTE:
                          the validator's index in vals                      */
  uint32_t n_verified; /* signatures sent to the device                      */
  uint32_t reserved;
} cmtv_commit_result;

/* VerifyCommit / VerifyCommitLight / VerifyCommitLightTrusting
 * (types/validator_set.go:667 / 722 / 775). Verifies every signature the
 * reference loop could reach in one device batch, then replays the reference
 * loop in index order over the verdicts, so the first error, the early exits
 * and the tallies are exactly the reference's. `msg_buf` (may be NULL)
 * receives the reference's error string (NUL-terminated, truncated to
 * msg_cap). trust_num/trust_den are only read for LIGHT_TRUSTING (the
 * validator set need not match the commit; matching is by address).
 * Returns CMTV_OK when the commit verifies, CMTV_ECOMMIT when the reference
 * would return an error (details in *res), another negative code on a
 * library failure. */
int cmtv_verify_commit(cmtv_ctx* ctx, uint32_t kind, uint32_t mode, const char* chain_id, size_t chain_id_len,
                       const cmtv_valset* vals, const cmtv_block_id* block_id, int64_t height,
                       const cmtv_commit* commit, uint64_t trust_num, uint64_t trust_den, cmtv_commit_result* res,
                       char* msg_buf, size_t msg_cap);

/* Cross-height batching (blocksync / light-client replay):
 * n commits, each with its own validator set, block ID and height, verified
 * with ONE device batch for all their signatures, then each commit's
 * reference loop replayed over its verdicts. Per commit i the outcome equals
 * cmtv_verify_commit(ctx, kind, mode, chain_id, vals[i], block_ids[i] (unused
 * for LIGHT_TRUSTING), heights[i], commits[i], ...): rcs[i] gets its return
 * code (CMTV_OK / CMTV_ECOMMIT), results[i] its details and msg_bufs +
 * i * msg_cap (may be NULL) its error string. Returns CMTV_OK when every
 * commit was evaluated, a negative library code otherwise. */
int cmtv_verify_commits(cmtv_ctx* ctx, uint32_t kind, uint32_t mode, const char* chain_id, size_t chain_id_len,
                        size_t n, const cmtv_valset* vals, const cmtv_block_id* block_ids, const int64_t* heights,
                        const cmtv_commit* commits, uint64_t trust_num, uint64_t trust_den,
                        cmtv_commit_result* results, int* rcs, char* msg_bufs, size_t msg_cap);

/* Pinned host memory for the caller's argument arena (the
 * zero-copy boundary). A cgo shim that builds its cmtv_verify_commits
 * arguments -- each commit's flags, ts_seconds, ts_nanos and signatures -- in
 * a block from cmtv_alloc_pinned lets the cross-height pipeline DMA them
 * straight to every device of the context: no host copy per signature
 * (cmtv_stats.direct_chunks counts such chunks). It applies to commits whose
 * reference loop reaches a prefix of their signatures (VerifyCommit: no
 * absent or unknown flags; VerifyCommitLight: no nil vote before +2/3), with
 * 64-byte signatures back to back and the registered-key cache on; any other
 * commit is packed as before, with identical outcomes. The block is
 * page-locked and portable to every device; the caller owns it, the library
 * reads it during calls only. Free it with cmtv_free_pinned on the same
 * context, never while a call that reads it runs (cmtv_close frees what is
 * left). Replaces: nothing in the reference (Go memory); INTEGRATION.md 4c
 * builds the blocksync window's arena in it. */
int cmtv_alloc_pinned(cmtv_ctx* ctx, size_t bytes, void** out);
int cmtv_free_pinned(cmtv_ctx* ctx, void* p);

/* CanonicalVote sign-bytes (types/vote.go:93 VoteSignBytes) for a commit
 * signature: writes up to cap bytes, returns the length (or negative code). */
int64_t cmtv_vote_sign_bytes(const char* chain_id, size_t chain_id_len, int32_t vote_type, int64_t height,
                             int32_t round, const cmtv_block_id* block_id, int64_t ts_seconds, int32_t ts_nanos,
                             uint8_t* out, size_t cap);

/* ------------------------------------------------------------ test-data generation */

/* RFC 8032 key generation and deterministic signing on the device (the
 * reference's crypto/ed25519 GenPrivKeyFromSecret / PrivKey.Sign,
 * ed25519.go:122,57), for synthetic validator sets and commits.
 * key_idx (optional): signature i uses seeds[key_idx[i]]. Blocking. */
int cmtv_pubkeys_ed25519(cmtv_ctx* ctx, size_t n, const uint8_t* seeds, uint8_t* out_pk);
int cmtv_sign_ed25519(cmtv_ctx* ctx, size_t n, const uint8_t* seeds, const uint32_t* key_idx, const uint8_t* msg,
                      const uint32_t* msg_off, uint8_t* out_sig);

#ifdef __cplusplus
}
#endif

#endif /* CMTVERIFY_H */
