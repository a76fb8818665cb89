// commit_internal.h -- the VerifyCommit* evaluation shared by the one-batch
// path (commit.cpp) and the chunked cross-height pipeline (pipeline.cpp):
// the CanonicalVote prefix encoder, the preamble + plan of a commit, and the
// reference loop replayed over device verdicts. Not part of the C ABI.
//
// Reference: types/validator_set.go:667-826 (VerifyCommit, VerifyCommitLight,
// VerifyCommitLightTrusting), types/block.go:652-665 (CommitSig.BlockID),
// types/vote.go:93 (VoteSignBytes), types/canonical.go:18-65,
// proto/tendermint/types/canonical.pb.go:517-567.
#pragma once
#include <hip/hip_runtime.h>  // signbytes.h: __host__ __device__
#include <stdint.h>
#include <stddef.h>

#include <algorithm>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cmtverify.h"
#include "signbytes.h"

namespace cmtv {

constexpr uint8_t kFlagAbsent = 1, kFlagCommit = 2, kFlagNil = 3;
constexpr int32_t kPrecommit = 2;

// ------------------------------------------------------------------ encoding

// Protobuf writer over a byte buffer; with p == nullptr it only counts, so
// one function gives both a field's length and its bytes (no temporaries).
struct ByteWriter {
  uint8_t* p = nullptr;
  size_t n = 0;
  void byte(uint8_t b) {
    if (p) p[n] = b;
    n++;
  }
  void bytes(const uint8_t* s, size_t len) {
    if (p && len) std::memcpy(p + n, s, len);
    n += len;
  }
  void uvarint(uint64_t v) {
    while (v >= 0x80) {
      byte((uint8_t)((v & 0x7F) | 0x80));
      v >>= 7;
    }
    byte((uint8_t)v);
  }
  void sfixed64(uint8_t tag, int64_t v) {
    byte(tag);
    const uint64_t u = (uint64_t)v;
    for (int i = 0; i < 8; i++) byte((uint8_t)(u >> (8 * i)));
  }
  void bytes_field(uint8_t tag, const uint8_t* s, size_t len) {
    byte(tag);
    uvarint(len);
    bytes(s, len);
  }
};

inline size_t uvarint_len(uint64_t v) { return sb_uvlen(v); }

inline bool block_id_is_zero(const cmtv_block_id* b) {
  return !b || (b->hash_len == 0 && b->psh_total == 0 && b->psh_hash_len == 0);
}

// CanonicalBlockID (canonical.pb.go:370) as field 4 of CanonicalVote, or
// nothing when the BlockID IsZero (canonical.go:18-33)
inline void put_canonical_block_id(ByteWriter& w, const cmtv_block_id* b) {
  if (block_id_is_zero(b)) return;
  const size_t psh = (b->psh_total ? 1 + uvarint_len(b->psh_total) : 0) +
                     (b->psh_hash_len ? 1 + uvarint_len(b->psh_hash_len) + b->psh_hash_len : 0);
  const size_t cb = (b->hash_len ? 1 + uvarint_len(b->hash_len) + b->hash_len : 0) + 1 + uvarint_len(psh) + psh;
  w.byte(0x22);
  w.uvarint(cb);
  if (b->hash_len) w.bytes_field(0x0A, b->hash, b->hash_len);
  w.byte(0x12);
  w.uvarint(psh);
  if (b->psh_total) {
    w.byte(0x08);
    w.uvarint(b->psh_total);
  }
  if (b->psh_hash_len) w.bytes_field(0x12, b->psh_hash, b->psh_hash_len);
}

// The CanonicalVote fields before the timestamp (type, height, round,
// BlockID unless nil): the per-commit part of a signature's sign-bytes.
inline void put_vote_prefix(ByteWriter& w, int32_t vtype, int64_t height, int32_t round, const cmtv_block_id* bid) {
  if (vtype != 0) {
    w.byte(0x08);
    w.uvarint((uint64_t)(int64_t)vtype);
  }
  if (height != 0) w.sfixed64(0x11, height);
  if (round != 0) w.sfixed64(0x19, (int64_t)round);
  put_canonical_block_id(w, bid);
}

// A commit's sign-bytes template (signbytes.h): pre(Commit) || pre(Nil) ||
// chain-id field, written at blob + at (or only counted with blob == null).
// Returns the bytes; t gets offsets relative to `at`'s blob.
inline size_t put_commit_template(uint8_t* blob, size_t at, const char* chain_id, size_t chain_id_len,
                                  const cmtv_commit* c, SbTemplate* t) {
  static const cmtv_block_id empty{};
  ByteWriter w{blob ? blob + at : nullptr, 0};
  put_vote_prefix(w, kPrecommit, c->height, c->round, &c->block_id);
  const size_t l1 = w.n;
  put_vote_prefix(w, kPrecommit, c->height, c->round, &empty);
  const size_t l2 = w.n - l1;
  if (chain_id_len) w.bytes_field(0x32, reinterpret_cast<const uint8_t*>(chain_id), chain_id_len);
  if (t) {
    t->pre_commit_off = (uint32_t)at;
    t->pre_commit_len = (uint32_t)l1;
    t->pre_nil_off = (uint32_t)(at + l1);
    t->pre_nil_len = (uint32_t)l2;
    t->post_off = (uint32_t)(at + l1 + l2);
    t->post_len = (uint32_t)(w.n - l1 - l2);
  }
  return w.n;
}

// put_commit_template's lengths without writing or counting byte by byte:
// the pre(Commit), pre(Nil) and chain-id field lengths; returns their sum
// (the template's blob bytes). The same numbers as put_commit_template's
// (tests/host/pipecheck.cpp compares them on every commit it plans).
inline size_t commit_template_lens(size_t chain_id_len, const cmtv_commit* c, uint32_t* pre_commit,
                                   uint32_t* pre_nil, uint32_t* post) {
  const cmtv_block_id* b = &c->block_id;
  const size_t base = 2 + (c->height != 0 ? 9 : 0) + (c->round != 0 ? 9 : 0);  // type, height, round
  size_t bid = 0;
  if (!block_id_is_zero(b)) {
    const size_t psh = (b->psh_total ? 1 + sb_uvlen(b->psh_total) : 0) +
                       (b->psh_hash_len ? 1 + sb_uvlen(b->psh_hash_len) + b->psh_hash_len : 0);
    const size_t cb = (b->hash_len ? 1 + sb_uvlen(b->hash_len) + b->hash_len : 0) + 1 + sb_uvlen(psh) + psh;
    bid = 1 + sb_uvlen(cb) + cb;
  }
  *pre_commit = (uint32_t)(base + bid);
  *pre_nil = (uint32_t)base;
  *post = (uint32_t)(chain_id_len ? 1 + sb_uvlen(chain_id_len) + chain_id_len : 0);
  return *pre_commit + *pre_nil + *post;
}

// sb_msg_len (signbytes.h) without loops or tables: a varint's length is
// ceil(bits / 7) (at least 1), and (bits + 6) / 7 == ((bits + 6) * 37) >> 8
// for every bits in 1..64 (checked exhaustively by tests/test_pipeline_cpu.py's
// host build: tests/host/pipecheck.cpp compares every message's offsets with
// sb_msg_len). Same value for every input.
inline uint32_t uvlen(uint64_t v) {
  const uint32_t bits = 64 - (uint32_t)__builtin_clzll(v | 1);
  return ((bits + 6) * 37) >> 8;
}

struct TplLens {
  uint32_t pre_commit, pre_nil, post;
};

inline uint32_t msg_len(const TplLens& t, bool commit_flag, int64_t sec, int32_t nanos) {
  // the timestamp is at most 22 bytes, so its length varint is one byte
  const uint32_t tl = (sec != 0 ? 1 + uvlen((uint64_t)sec) : 0) + (nanos != 0 ? 1 + uvlen((uint64_t)(int64_t)nanos) : 0);
  const uint32_t b = (commit_flag ? t.pre_commit : t.pre_nil) + 2 + tl + t.post;
  return b + (b < 128 ? 1 : uvlen(b));
}

// the longest message a template can give (a 22-byte timestamp)
inline uint32_t msg_len_bound(const TplLens& t) {
  const uint32_t b = std::max(t.pre_commit, t.pre_nil) + 2 + 22 + t.post;
  return b + uvlen(b);
}

// ------------------------------------------------------------------ formatting

inline std::string hex_upper(const uint8_t* p, size_t n) {
  static const char* d = "0123456789ABCDEF";
  std::string s;
  s.reserve(2 * n);
  for (size_t i = 0; i < n; i++) {
    s.push_back(d[p[i] >> 4]);
    s.push_back(d[p[i] & 15]);
  }
  return s;
}

inline void set_msg(char* buf, size_t cap, const std::string& s) {
  if (!buf || cap == 0) return;
  size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
  std::memcpy(buf, s.data(), n);
  buf[n] = 0;
}

// ------------------------------------------------------------------ lookups

// ValidatorSet.GetByAddress (validator_set.go:270-277: the first validator
// with that address) as an open-addressing table over 20-byte addresses,
// hashed with a per-process key (the looked-up addresses come from peers).
struct AddrIndex {
  const uint8_t* addrs = nullptr;
  std::vector<uint32_t> slot;  // validator index + 1; 0 = empty
  uint64_t mask = 0;
  static uint64_t key();
  static uint64_t hash(const uint8_t* a) {
    uint64_t x, y;
    std::memcpy(&x, a, 8);
    std::memcpy(&y, a + 8, 8);
    x ^= key();
    x = (x ^ (y * 0x9E3779B97F4A7C15ull)) * 0xBF58476D1CE4E5B9ull;
    return x ^ (x >> 31);
  }
  void build(const uint8_t* a, uint32_t n) {
    addrs = a;
    size_t cap = 16;
    while (cap < 2 * (size_t)n) cap <<= 1;
    slot.assign(cap, 0);
    mask = cap - 1;
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t* p = a + 20 * (size_t)i;
      for (uint64_t h = hash(p) & mask;; h = (h + 1) & mask) {
        if (slot[h] == 0) {
          slot[h] = i + 1;
          break;
        }
        if (std::memcmp(addrs + 20 * (size_t)(slot[h] - 1), p, 20) == 0) break;  // first wins
      }
    }
  }
  // validator index or -1
  int64_t find(const uint8_t* p) const {
    for (uint64_t h = hash(p) & mask;; h = (h + 1) & mask) {
      if (slot[h] == 0) return -1;
      if (std::memcmp(addrs + 20 * (size_t)(slot[h] - 1), p, 20) == 0) return (int64_t)slot[h] - 1;
    }
  }
};

// The double-vote map of VerifyCommitLightTrusting (validator_set.go:805):
// validator index -> first commit index, reset in O(1) per commit by epoch.
struct Seen {
  std::vector<uint32_t> stamp, first;
  uint32_t epoch = 0;
  void reset(uint32_t n_vals) {
    if (stamp.size() < n_vals) {
      stamp.assign(n_vals, 0);
      first.assign(n_vals, 0);
      epoch = 0;
    }
    if (++epoch == 0) {
      std::fill(stamp.begin(), stamp.end(), 0);
      epoch = 1;
    }
  }
  bool has(uint32_t vi, uint32_t* f) const {
    if (stamp[vi] != epoch) return false;
    *f = first[vi];
    return true;
  }
  void put(uint32_t vi, uint32_t idx) {
    stamp[vi] = epoch;
    first[vi] = idx;
  }
};

// ------------------------------------------------------------------ one commit

// One VerifyCommit* evaluation: preamble, plan (the signatures the
// reference loop can reach), then the loop replayed over device verdicts.
struct CommitJob {
  uint32_t kind;
  const char* chain_id;
  size_t chain_id_len;
  const cmtv_valset* vals;
  const cmtv_block_id* block_id;
  int64_t height;
  const cmtv_commit* commit;
  uint64_t trust_num, trust_den;
  cmtv_commit_result* res;
  char* msg_buf;
  size_t msg_cap;
  // state
  int early = 1;  // != 1: the preamble already decided (return code)
  int64_t needed = 0;
  const AddrIndex* addr = nullptr;  // LightTrusting: index of vals' addresses
  std::vector<uint32_t> plan_idx, plan_val;
  size_t first = 0;  // batch index of plan item 0
  size_t plan_prefix = 0;  // > 0: the plan is signatures [0, plan_prefix) (plan_idx unused)
  int64_t prefix_tally = 0;  // ... and the tally the loop reaches over it when every verdict is valid
  // the validator set's total voting power when the caller already has it
  // (the pipeline: one sum per distinct set, not per commit)
  bool has_total = false;
  int64_t total = 0;

  int fail(int32_t code, int32_t idx, const std::string& m) {
    res->code = code;
    res->sig_index = idx;
    set_msg(msg_buf, msg_cap, m);
    return CMTV_ECOMMIT;
  }
};

// "wrong signature (#%d): %X" (validator_set.go:697, 753, 814)
inline int fail_wrong_sig(CommitJob& J, uint32_t idx) {
  const uint32_t s0 = J.commit->sig_off[idx], s1 = J.commit->sig_off[idx + 1];
  return J.fail(CMTV_COMMIT_ERR_WRONG_SIGNATURE, (int32_t)idx,
                "wrong signature (#" + std::to_string(idx) + "): " + hex_upper(J.commit->sigs + s0, s1 - s0));
}

// ErrNotEnoughVotingPowerSigned (validator_set.go:856-863)
inline int fail_not_enough(CommitJob& J, int64_t tally) {
  J.res->got = tally;
  J.res->needed = J.needed;
  char b[160];
  std::snprintf(b, sizeof b, "invalid commit -- insufficient voting power: got %" PRId64 ", needed more than %" PRId64,
                tally, J.needed);
  return J.fail(CMTV_COMMIT_ERR_NOT_ENOUGH_POWER, -1, b);
}

// The reference loop over a prefix plan (every signature [0, m) reachable,
// every flag, key and signature length already checked -- commit.cpp
// job_prepare_fast, pipeline.cpp direct commits): its outcome is the first
// invalid verdict first_bad (m: none), else the tally against the threshold
// (job_replay gives the same, one signature at a time).
inline int replay_prefix(CommitJob& J, size_t m, int64_t tally, size_t first_bad) {
  if (J.early != 1) return J.early;
  J.res->n_verified = (uint32_t)m;
  if (first_bad < m) return fail_wrong_sig(J, (uint32_t)first_bad);
  return tally > J.needed ? CMTV_OK : fail_not_enough(J, tally);
}

// Argument checks of one commit (CMTV_EINVAL on null arrays).
int job_check_args(uint32_t kind, const char* chain_id, size_t chain_id_len, const cmtv_valset* vals,
                   const cmtv_block_id* block_id, const cmtv_commit* commit, cmtv_commit_result* res);
// Resets *res, checks sizes / height / BlockID or the trust level and sets
// J.needed (validator_set.go:670-684, 779-790); J.early != 1 when decided.
// LightTrusting needs J.addr set.
void job_preamble(CommitJob& J);
// The plan (validator_set.go:685-707, 740-762, 793-823 assuming every
// verdict valid): writes commit indices to pidx and validator indices to
// pval (pval may be null unless LightTrusting); returns its length
// (<= commit->n_sigs).
size_t job_plan(const CommitJob& J, uint32_t* pidx, uint32_t* pval, Seen& seen);

// The reference loop (validator_set.go:685-713, 740-764, 793-825) over the
// verdicts of the m planned signatures pidx[0..m) (pidx null: the plan is
// the commit's first m signatures): valid(j) is plan item j's
// device verdict; a signature whose length is not 64 is invalid whatever the
// device said, and fails before its key's length is looked at
// (crypto/ed25519/ed25519.go:150).
template <class V>
int job_replay(CommitJob& J, const uint32_t* pidx, size_t m, V valid, Seen& seen) {
  if (J.early != 1) return J.early;
  const cmtv_valset* vals = J.vals;
  const cmtv_commit* commit = J.commit;
  const uint32_t nsig = commit->n_sigs;
  J.res->n_verified = (uint32_t)m;
  // PubKey.VerifySignature (crypto/ed25519/ed25519.go:148-155) returns false
  // for a signature that is not 64 bytes BEFORE Go's ed25519.Verify can panic
  // on a key that is not 32 bytes
  auto sig64 = [&](uint32_t idx) { return commit->sig_off[idx + 1] - commit->sig_off[idx] == 64; };
  auto wrong_sig = [&](uint32_t idx) { return fail_wrong_sig(J, idx); };
  auto bad_pk = [&](uint32_t idx, uint32_t vi) {
    return J.fail(CMTV_COMMIT_PANIC_BAD_PUBKEY, (int32_t)idx,
                  "ed25519: bad public key length: " + std::to_string(vals->pk_off[vi + 1] - vals->pk_off[vi]));
  };
  int64_t tally = 0;
  size_t j = 0;
  if (J.kind == CMTV_VERIFY_COMMIT_LIGHT_TRUSTING) seen.reset(vals->n_vals);
  for (uint32_t idx = 0; idx < nsig; idx++) {
    const uint8_t flag = commit->flags[idx];
    if (J.kind == CMTV_VERIFY_COMMIT) {
      if (flag == kFlagAbsent) continue;
      if (flag != kFlagCommit && flag != kFlagNil)
        return J.fail(CMTV_COMMIT_PANIC_UNKNOWN_FLAG, (int32_t)idx, "Unknown BlockIDFlag: " + std::to_string(flag));
      if (!sig64(idx)) return wrong_sig(idx);
      if (vals->pk_off[idx + 1] - vals->pk_off[idx] != 32) return bad_pk(idx, idx);
      if (j >= m || (pidx ? pidx[j] : (uint32_t)j) != idx || !valid(j)) return wrong_sig(idx);
      j++;
      if (flag == kFlagCommit) tally += vals->voting_power[idx];
    } else {
      if (flag != kFlagCommit) continue;
      uint32_t vi = idx;
      if (J.kind == CMTV_VERIFY_COMMIT_LIGHT_TRUSTING) {
        const int64_t f = J.addr->find(commit->val_addrs + 20 * (size_t)idx);
        if (f < 0) continue;
        vi = (uint32_t)f;
        uint32_t first = 0;
        if (seen.has(vi, &first)) {
          // Validator.String(): "Validator{%v %v VP:%v A:%v}" (types/validator.go)
          std::string vs = "Validator{" + hex_upper(vals->addrs + 20 * (size_t)vi, 20) + " PubKeyEd25519{" +
                           hex_upper(vals->pubkeys + vals->pk_off[vi], vals->pk_off[vi + 1] - vals->pk_off[vi]) +
                           "} VP:" + std::to_string(vals->voting_power[vi]) + " A:" +
                           std::to_string(vals->proposer_priority ? vals->proposer_priority[vi] : 0) + "}";
          // the Go side formats the error with its own Validator: got = the
          // first commit index, needed = the validator's index in vals
          J.res->got = first;
          J.res->needed = vi;
          return J.fail(CMTV_COMMIT_ERR_DOUBLE_VOTE, (int32_t)idx,
                        "double vote from " + vs + " (" + std::to_string(first) + " and " + std::to_string(idx) +
                            ")");
        }
        seen.put(vi, idx);
      }
      if (!sig64(idx)) return wrong_sig(idx);
      if (vals->pk_off[vi + 1] - vals->pk_off[vi] != 32) return bad_pk(idx, vi);
      if (j >= m || (pidx ? pidx[j] : (uint32_t)j) != idx || !valid(j)) return wrong_sig(idx);
      j++;
      tally += vals->voting_power[vi];
      if (tally > J.needed) return CMTV_OK;
    }
  }
  if (J.kind == CMTV_VERIFY_COMMIT && tally > J.needed) return CMTV_OK;
  return fail_not_enough(J, tally);
}

// Two validator sets hold the same keys (one registered key set serves both).
bool same_keys(const cmtv_valset* a, const cmtv_valset* b);

// The arguments of one cmtv_verify_commits call (checked by the caller).
struct CommitsArgs {
  uint32_t kind, mode;
  const char* chain_id;
  size_t chain_id_len, n;
  const cmtv_valset* vals;
  const cmtv_block_id* block_ids;  // null for LightTrusting
  const int64_t* heights;
  const cmtv_commit* commits;
  uint64_t trust_num, trust_den;
  cmtv_commit_result* results;
  char* msg_bufs;
  size_t msg_cap;
  CommitJob job(size_t c) const {
    return CommitJob{kind, chain_id, chain_id_len, &vals[c], block_ids ? &block_ids[c] : nullptr, heights[c],
                     &commits[c], trust_num, trust_den, &results[c], msg_bufs ? msg_bufs + c * msg_cap : nullptr,
                     msg_bufs ? msg_cap : 0};
  }
};

// The chunked cross-height pipeline (pipeline.cpp): fills rcs[0..a.n).
// Returns CMTV_OK or a library error. Used by cmtv_verify_commits for large
// calls without the verdict cache.
int verify_commits_pipeline(cmtv_ctx* ctx, const CommitsArgs& a, int* rcs);
// Whether cmtv_verify_commits takes the pipeline for a call of this many
// signatures (CMTV_PIPE_MIN).
bool pipeline_wanted(const cmtv_ctx* ctx, uint64_t n_sigs);
// Largest sign-bytes span of one device launch (its message offsets are
// 32-bit): 2^31, or CMTV_MAX_BATCH_MSG_BYTES when lower (commit.cpp).
uint64_t max_batch_msg_bytes();

}  // namespace cmtv
