// Host-side fixed-base table for the quad/oct verifiers' checks: rows of the
// device B table (verify_core.h: three radix-256 blocks, then the three
// (1..2^15)[2^shift]B radix-2^16 blocks) computed on first use, since a
// host build of all 98,688 rows would take minutes. Thread-safe (quadcheck
// runs the four lanes of a quad as threads). Test infrastructure.
#pragma once
#include <array>
#include <mutex>
#include <unordered_map>

#include "../../cometbft_amd/csrc/verify_core.h"

namespace cmtv {

struct LazyBTab {
  mutable std::mutex mu;
  mutable std::unordered_map<int, std::array<uint32_t, BTAB_ROW_WORDS>> rows;
  const uint32_t* row(int e) const {
    std::lock_guard<std::mutex> g(mu);
    auto it = rows.find(e);
    if (it == rows.end()) {
      std::array<uint32_t, BTAB_ROW_WORDS> r{};
      if (e < BT16_BASE) {
        btab_entry(r.data(), e % BTAB_ENTRIES + 1, e / BTAB_ENTRIES);
      } else {
        const int f = e - BT16_BASE;
        btab_entry_shift(r.data(), f % BT16_ENTRIES + 1, bt16_block_shift(f / BT16_ENTRIES), 16);
      }
      it = rows.emplace(e, r).first;
    }
    return it->second.data();
  }
  void load_coord(int e, int off, fe& r) const {
    const uint32_t* p = row(e) + off;
    for (int i = 0; i < 10; i++) r.v[i] = p[i];
  }
};

}  // namespace cmtv
