// kernels.h -- host-side launchers for the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmtv {

// (1..128)B, [2^124]B, [2^128]B multiples, then (1..2^15)B, [2^120]B, [2^128]B
// multiples, then the 16-position comb (1..2^15)[2^16j]B (verify_core.h
// BTAB_TOTAL_ROWS); 36 words per row, 89.7 MB
constexpr uint32_t kBtabWords = (3 * 128 + 3 * 32768 + 16 * 32768) * 36;
constexpr uint32_t kAtabWordsPerLane = 320; // (1..8)(-A), 40 words per point
constexpr uint32_t kCombWords = 32 * 128 * 32;     // one registered-key comb (keyed.h), 512 KiB
constexpr uint32_t kCombScratchWordsPerKey = 128 * 320;  // prefix products while building

// The verification forms (launch_verify / launch_verify_sr25519 kflags bits
// 0..7; the runtime picks one per batch size, runtime.cpp ed_form / sr_form):
//   kFormLane : one signature per lane (k_verify, k_verify_sr25519)
//   kFormQuad : four lanes per signature, three quad waves + a helper wave
//               that hashes and sums each window's table entries
//               (k_verify_quad_hs, k_verify_sr25519_quad_hs)
//   kFormOct2 : eight lanes per signature in two waves (k_verify_oct_split)
//   kFormRow  : one wave per signature, three per workgroup + a helper
//               (k_verify_row_split)
//   kFormRow4 : four waves per signature (k_verify_row4_split)
// sr25519 has the lane and quad forms. kLaunchForceWide: the CMTV_FORCE_WIDE
// test knob (every quad-family verifier takes the 64-window schedule); bits
// 16..31: the helper-summed forms' tuning (hs_tune, CMTV_HS_PRE).
constexpr uint32_t kFormLane = 0, kFormQuad = 1, kFormOct2 = 2, kFormRow = 3, kFormRow4 = 4;
constexpr uint32_t kFormMask = 0xFF, kLaunchForceWide = 0x100;
// registered-key forms (launch_verify_keyed): the keyed row kernel
// (k_verify_keyed_row_split, one signature per workgroup), the keyed quad
// kernel with two helper waves (k_verify_keyed_quad_split), the lane kernels
// (keyed_lane.hip)
constexpr uint32_t kKeyedRow = 0, kKeyedQuad = 1, kKeyedLane = 2;

// Row kernel bitmap assembly: each launch takes the next of kRowSlots slots
// of a per-device ring (kRowSlotWords words, read as 64-bit words of 32
// two-bit verdict fields: kernels.hip row_bitmap_add); the wave that fills a
// word's last field writes that word's 32 bitmap bits and zeroes it. A slot is
// reused after kRowSlots further row launches on the device; the runtime
// fences a reuse against the slot's previous launch (runtime.cpp
// row_slot_acquire). kRowMaxCap bounds a row launch.
constexpr uint32_t kRowSlots = 256, kRowSlotWords = 1024, kRowMaxCap = 4 * (kRowSlotWords - 16);
// A row launch's ring slot and, optionally, its tagged bitmap: with tagged
// set (a device pointer to mapped host memory, one entry per 32 signatures),
// the wave that completes word j stores (seq << 32 | the word's 32 bits) into
// tagged[j] with ONE 64-bit system-scope atomic store instead of writing the
// bitmap, so the host knows the bitmap is complete when every entry carries
// seq -- without waiting for the kernel to retire, and without any ordering
// between the waves' stores (runtime.cpp wait_row_tags). The slot word is zero
// again before its entry is stored.
struct RowSlot {
  uint32_t* words = nullptr;
  uint64_t* tagged = nullptr;
  uint32_t seq = 0;
};

// Templated sign-bytes (signbytes.h) written by the helper waves of the
// helper-wave kernels themselves (every form but the lane kernels): each
// helper lane builds its signature's CanonicalVote into an LDS slot of
// kSbFuseMaxMsg bytes and hashes it from there, so a templated commit needs
// no k_sign_bytes launch (and no global message buffer). Device pointers;
// tmpls == nullptr means the messages are in `msg`.
struct SbFuse {
  const void* tmpls = nullptr;
  const uint8_t* blob = nullptr;
  const uint32_t* tidx = nullptr;
  const uint8_t* flag = nullptr;
  const int64_t* sec = nullptr;
  const int32_t* nanos = nullptr;
};
constexpr uint32_t kSbFuseMaxMsg = 192;

// Per-device diagnostic counters the kernels bump with vector atomics
// (CmtvDev::d_diag, read by cmtv_stats_get): kDiagLateK = quad waves of
// k_verify_keyed_quad_split that stopped waiting for the hash helper and
// hashed their own signatures. kKeyedWaitDefault = the polls before that.
constexpr uint32_t kDiagLateK = 0, kDiagWords = 4;
constexpr uint32_t kKeyedWaitDefault = 1u << 22;

hipError_t launch_btab_init(uint32_t* d_rows, hipStream_t s);
// sb (may be null) is honoured by the forms whose helper wave hashes (every
// form but kFormLane); the caller launches k_sign_bytes otherwise. The row
// forms need row_slot (one slot of the device's ring) when bitmap is set.
hipError_t launch_verify(uint32_t mode, uint32_t n, const void* pk, const void* sig, const void* msg,
                         const void* off, const uint32_t* btab, uint32_t* atab, void* valid, void* bitmap,
                         uint32_t kflags, hipStream_t s, const SbFuse* sb = nullptr, const RowSlot* row_slot = nullptr);
hipError_t launch_comb_build(uint32_t n_keys, const void* keys_pk, uint8_t* keys_ok, uint32_t* tabs,
                             uint32_t* scratch, bool negate, hipStream_t s);
// form: kKeyedRow (row_slot: a slot of the device's bitmap ring when bitmap
// is set), kKeyedQuad, kKeyedLane. sb (may be null) is honoured by the row and
// quad forms only (their helper waves hash; hipErrorInvalidValue otherwise).
// key_idx null: signature i is by key i (row and quad forms).
hipError_t launch_verify_keyed(uint32_t mode, uint32_t n, uint32_t n_keys, const void* key_idx, const void* sig,
                               const void* msg, const void* off, const uint32_t* keys_pk, const uint8_t* keys_ok,
                               const uint32_t* ktabs, void* valid, void* bitmap, uint32_t form, uint32_t k_wait,
                               uint32_t* diag, uint32_t batch_kb, uint32_t* scr, const uint32_t* wtabs,
                               const uint32_t* btab, hipStream_t s, const RowSlot* row_slot = nullptr,
                               const SbFuse* sb = nullptr);
// the one-signature-per-lane part of launch_verify_keyed (keyed_lane.hip):
// over the wide combs wtabs (rows staged by LDS-DMA) or, with wtabs null, the
// radix-256 key combs ktabs with B over btab's radix-2^16 comb
hipError_t launch_verify_keyed_lane(uint32_t mode, uint32_t n, uint32_t n_keys, const uint32_t* ki,
                                    const uint32_t* sgp, const uint8_t* mp, const uint32_t* op,
                                    const uint32_t* keys_pk, const uint8_t* keys_ok, const uint32_t* ktabs,
                                    uint8_t* vp, uint64_t* bp, uint32_t batch_kb, uint32_t* scr,
                                    const uint32_t* wtabs, const uint32_t* btab, hipStream_t s);
// Wide (radix-2^16) combs of n_keys keys (keyed.h): bases = n_keys x 16 x 40
// words, scratch = n_keys x kWideScratchWordsPerKey words.
constexpr size_t kWideTableWords = (size_t)16 * 32768 * 32;  // 64 MiB per key
constexpr size_t kWideScratchWordsPerKey = (size_t)16 * (32768 / 64) * 64 * 10;
constexpr size_t kWideBaseWordsPerKey = 16 * 40;
hipError_t launch_wide_build(uint32_t n_keys, const void* keys_pk, uint32_t* tabs, uint32_t* bases,
                             uint32_t* scratch, hipStream_t s);
// k_verify_keyed_batch: signatures per lane, and its scratch per lane
// (kb x 40 words: R'.X and R'.Y (Go) or the coset x numerator (ZIP-215), Z,
// and the running product of the Z's)
constexpr uint32_t kKeyedBatchScratchWordsPerSig = 40;
hipError_t launch_verify_sr25519(uint32_t n, const void* pk, const void* sig, const void* msg, const void* off,
                                 const uint32_t* btab, uint32_t* atab, const uint32_t* prog, int nops, void* valid,
                                 void* bitmap, uint32_t kflags, hipStream_t s);
hipError_t launch_sign_bytes(uint32_t n, const void* tmpls, const uint8_t* blob, const uint32_t* tidx,
                             const uint8_t* commit_flag, const int64_t* sec, const int32_t* nanos,
                             const uint32_t* off, uint8_t* msg, hipStream_t s);
// direct cross-height chunks (signbytes.hip): n_c commits (BulkDesc, their
// templates) whose arrays sit in `arena` (the chunk's device copy of the
// caller's pinned memory) -> the per-signature chunk layout of m planned
// signatures and their message offsets (off[0..m]); ctot / cbase: n_c words
// each of scratch
hipError_t launch_bulk_gather(uint32_t n_c, uint32_t m, const void* desc, const void* tmpls, const uint8_t* arena,
                              uint32_t* kidx, uint8_t* sig, uint32_t* off, uint32_t* tidx, uint8_t* flag,
                              int64_t* sec, int32_t* nanos, uint32_t* ctot, uint32_t* cbase, hipStream_t s);
hipError_t launch_pubkey(uint32_t n, const void* seeds, const uint32_t* btab, void* out_pk, hipStream_t s);
hipError_t launch_sign(uint32_t n, const void* seeds, const void* key_idx, const void* msg, const void* off,
                       const uint32_t* btab, void* out_sig, hipStream_t s);

}  // namespace cmtv
