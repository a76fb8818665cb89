// signbytes.h -- CanonicalVote sign-bytes from a per-commit template
// (device-side sign-bytes templating).
//
// VoteSignBytes (/root/reference/types/vote.go:93-101) of a commit signature
// is uvarint(len(body)) || body with body the CanonicalVote
// (proto/tendermint/types/canonical.pb.go:517-567):
//
//   pre(flag)  type, height, round, CanonicalBlockID (present for
//              BlockIDFlagCommit, omitted for BlockIDFlagNil: CommitSig.BlockID,
//              types/block.go:652-665)                       -- per commit
//   0x2A uvarint(len(ts)) ts,  ts = [0x08 uvarint(sec)] [0x10 uvarint(nanos)]
//              (gogoproto StdTime; zero fields omitted)      -- per signature
//   post       0x32 uvarint(len(chain_id)) chain_id          -- per chain
//
// Everything but the timestamp and the flag is shared by a commit's
// signatures, so the host ships one template per commit and 13 bytes per
// signature; the device writes the message bytes (k_sign_bytes). Lengths
// (and so the message offsets) are computed on both sides by the same
// functions below.
#pragma once
#include <stdint.h>

#ifndef CMTV_HD
#define CMTV_HD __host__ __device__ __forceinline__
#endif

namespace cmtv {

// template header: byte ranges inside the template byte blob
struct SbTemplate {
  uint32_t pre_commit_off, pre_commit_len;  // type/height/round/BlockID
  uint32_t pre_nil_off, pre_nil_len;        // type/height/round
  uint32_t post_off, post_len;              // chain id field
};

// One commit of a direct cross-height chunk (pipeline.cpp with the caller's
// arguments in cmtv_alloc_pinned memory; runtime.cpp bulk_submit_locked;
// k_bulk_gather): where the commit's arrays landed in the chunk's device copy
// of the caller's pinned arena (byte offsets), and its plan, which is the
// commit's signatures [0, m) -- batch indices [sp, sp + m). Its template and
// commit index is its position in the chunk.
struct BulkDesc {
  uint64_t sig;    // signature 0 (64-byte records, 8-byte aligned)
  uint64_t sec;    // ts_seconds[0] (8-byte aligned)
  uint64_t nanos;  // ts_nanos[0] (4-byte aligned)
  uint64_t flags;  // flags[0]
  uint32_t sp, m;
};

CMTV_HD uint32_t sb_uvlen(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}

CMTV_HD uint32_t sb_ts_len(int64_t sec, int32_t nanos) {
  uint32_t n = 0;
  if (sec != 0) n += 1 + sb_uvlen((uint64_t)sec);
  if (nanos != 0) n += 1 + sb_uvlen((uint64_t)(int64_t)nanos);
  return n;
}

// body length (without the leading uvarint)
CMTV_HD uint32_t sb_body_len(const SbTemplate& t, bool commit_flag, int64_t sec, int32_t nanos) {
  const uint32_t tl = sb_ts_len(sec, nanos);
  return (commit_flag ? t.pre_commit_len : t.pre_nil_len) + 1 + sb_uvlen(tl) + tl + t.post_len;
}

CMTV_HD uint32_t sb_msg_len(const SbTemplate& t, bool commit_flag, int64_t sec, int32_t nanos) {
  const uint32_t b = sb_body_len(t, commit_flag, sec, nanos);
  return sb_uvlen(b) + b;
}

// writes uvarint(v) at out[pos..]; returns the new position
template <class Out>
CMTV_HD uint32_t sb_put_uvarint(Out& out, uint32_t pos, uint64_t v) {
  while (v >= 0x80) {
    out.put(pos++, (uint8_t)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  out.put(pos++, (uint8_t)v);
  return pos;
}

// The whole message of one signature. Out: put(pos, byte) and
// copy(pos, src, len) (the template's byte runs).
template <class Out>
CMTV_HD uint32_t sb_write(Out& out, const SbTemplate& t, const uint8_t* blob, bool commit_flag, int64_t sec,
                          int32_t nanos) {
  uint32_t pos = sb_put_uvarint(out, 0, sb_body_len(t, commit_flag, sec, nanos));
  const uint32_t po = commit_flag ? t.pre_commit_off : t.pre_nil_off;
  const uint32_t pl = commit_flag ? t.pre_commit_len : t.pre_nil_len;
  out.copy(pos, blob + po, pl);
  pos += pl;
  out.put(pos++, 0x2A);
  pos = sb_put_uvarint(out, pos, sb_ts_len(sec, nanos));
  if (sec != 0) {
    out.put(pos++, 0x08);
    pos = sb_put_uvarint(out, pos, (uint64_t)sec);
  }
  if (nanos != 0) {
    out.put(pos++, 0x10);
    pos = sb_put_uvarint(out, pos, (uint64_t)(int64_t)nanos);
  }
  out.copy(pos, blob + t.post_off, t.post_len);
  return pos + t.post_len;
}

}  // namespace cmtv
