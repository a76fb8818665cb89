// Host-side fixed-base table for the quad/oct verifiers' checks: rows of the
// device B table (verify_core.h btab_row: every block) computed on first
// use, since a host build of all 622,976 rows would take far too long. Thread-safe (quadcheck
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
      btab_row(r.data(), e);
      it = rows.emplace(e, r).first;
    }
    return it->second.data();
  }
  void load_coord(int e, int off, fe& r) const {
    const uint32_t* p = row(e) + off;
    for (int i = 0; i < 10; i++) r.v[i] = p[i];
  }
  // the one-lane policy (ge_add_table): niels coordinate c of row e
  void load_fe(int e, int c, fe& r) const { load_coord(e, c * BTAB_COORD_WORDS, r); }
};

}  // namespace cmtv
