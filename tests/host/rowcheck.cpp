// Host emulation of the one-signature-per-wave "row" verifier
// (cometbft_amd/csrc/row.h): the kernel source runs on 64-lane arrays, DPP
// row moves and row exchanges are array permutations, and the operand bounds
// row.h states are asserted on every product. The scalars and [u]B come from
// q_prepare / q_bcomb16 as k_verify_row_split's helper wave computes them.
// Test infrastructure only.
//   stdin:  u32 n, then n records { u8 mode, pk[32], sig[64], u32 mlen, msg }
//   stdout: n verdict bytes
//   argv[1] == "mul": instead, random products / squarings / canonical tests
//   against a big-int reference (prints "ok" or the first mismatch)
#define CMTV_HD inline
#define CMTV_BOUNDS_CHECK 1
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../cometbft_amd/csrc/keyed_quad.h"
#include "../../cometbft_amd/csrc/row.h"
#include "lazy_btab.h"
#include <map>
#include <string>

namespace hostlv {

// one value per lane of a 64-lane wave
template <class T>
struct LV {
  T a[64];
  LV() { for (auto& x : a) x = T(); }
  LV(T v) { for (auto& x : a) x = v; }  // NOLINT: a uniform value on every lane
  T& operator[](int i) { return a[i]; }
  const T& operator[](int i) const { return a[i]; }
};
using U = LV<uint32_t>;
using U64 = LV<uint64_t>;
using B = LV<bool>;

#define LV_BIN(op)                                                                       \
  template <class T>                                                                     \
  LV<T> operator op(const LV<T>& x, const LV<T>& y) {                                    \
    LV<T> r;                                                                             \
    for (int i = 0; i < 64; i++) r.a[i] = x.a[i] op y.a[i];                              \
    return r;                                                                            \
  }                                                                                      \
  template <class T, class S>                                                            \
  LV<T> operator op(const LV<T>& x, S y) {                                               \
    LV<T> r;                                                                             \
    for (int i = 0; i < 64; i++) r.a[i] = x.a[i] op (T)y;                                \
    return r;                                                                            \
  }
LV_BIN(+)
LV_BIN(-)
LV_BIN(*)
LV_BIN(&)
LV_BIN(|)
LV_BIN(^)
LV_BIN(>>)
LV_BIN(<<)
#undef LV_BIN
template <class T>
LV<T> operator~(const LV<T>& x) {
  LV<T> r;
  for (int i = 0; i < 64; i++) r.a[i] = ~x.a[i];
  return r;
}
#define LV_CMP(op)                                                                       \
  template <class T>                                                                     \
  B operator op(const LV<T>& x, const LV<T>& y) {                                        \
    B r;                                                                                 \
    for (int i = 0; i < 64; i++) r.a[i] = x.a[i] op y.a[i];                              \
    return r;                                                                            \
  }                                                                                      \
  template <class T, class S>                                                            \
  B operator op(const LV<T>& x, S y) {                                                   \
    B r;                                                                                 \
    for (int i = 0; i < 64; i++) r.a[i] = x.a[i] op (T)y;                                \
    return r;                                                                            \
  }
LV_CMP(==)
LV_CMP(!=)
LV_CMP(<)
#undef LV_CMP
inline B operator||(const B& x, const B& y) {
  B r;
  for (int i = 0; i < 64; i++) r.a[i] = x.a[i] || y.a[i];
  return r;
}
inline B operator&&(const B& x, const B& y) {
  B r;
  for (int i = 0; i < 64; i++) r.a[i] = x.a[i] && y.a[i];
  return r;
}

static void fail(const char* what) {
  fprintf(stderr, "row bound violated: %s\n", what);
  abort();
}

inline U64 widen(const U& x) {
  U64 r;
  for (int i = 0; i < 64; i++) r.a[i] = x.a[i];
  return r;
}
inline U64 mad64(const U& a, const U& b, const U64& c) {
  U64 r;
  for (int i = 0; i < 64; i++) {
    const unsigned __int128 v = (unsigned __int128)a.a[i] * b.a[i] + c.a[i];
    if (v >> 64) fail("mad64 overflow");
    r.a[i] = (uint64_t)v;
  }
  return r;
}
inline U lo32(const U64& x) {
  U r;
  for (int i = 0; i < 64; i++) r.a[i] = (uint32_t)x.a[i];
  return r;
}
// the carries of a product's column sums: the first must fit 32 bits
inline U shr64(const U64& x, int s) {
  U r;
  for (int i = 0; i < 64; i++) {
    if ((x.a[i] >> s) >> 32) fail("carry above 2^32 (column sum >= 2^48)");
    r.a[i] = (uint32_t)(x.a[i] >> s);
  }
  return r;
}
// the high word of a column sum: the sum must be below 2^48
inline U hi32(const U64& x) {
  U r;
  for (int i = 0; i < 64; i++) {
    if (x.a[i] >> 48) fail("column sum >= 2^48");
    r.a[i] = (uint32_t)(x.a[i] >> 32);
  }
  return r;
}
inline U mul24(const U& a, const U& b) {
  U r;
  for (int i = 0; i < 64; i++) {
    if (a.a[i] >> 24 || b.a[i] >> 24) fail("mul24 operand >= 2^24");
    r.a[i] = a.a[i] * b.a[i];
  }
  return r;
}
template <class T>
LV<T> sel(const B& c, const LV<T>& x, const LV<T>& y) {
  LV<T> r;
  for (int i = 0; i < 64; i++) r.a[i] = c.a[i] ? x.a[i] : y.a[i];
  return r;
}

// the row policy
struct HostRow {
  using U = hostlv::U;
  using U64 = hostlv::U64;
  using B = hostlv::B;
  static constexpr bool kFusedProduct = false;
  static U lane() {
    U r;
    for (int i = 0; i < 64; i++) r.a[i] = i;
    return r;
  }
  template <int R>
  static U ror(const U& x) {
    U r;
    for (int i = 0; i < 64; i++) r.a[i] = x.a[(i & ~15) | ((i - R) & 15)];
    return r;
  }
  template <int R>
  static U bcast(const U& x) {
    U r;
    for (int i = 0; i < 64; i++) r.a[i] = x.a[(i & ~15) | R];
    return r;
  }
  static void rows(const U& x, U& b0, U& b1, U& b2, U& b3) {
    for (int i = 0; i < 64; i++) {
      const int k = i & 15;
      b0.a[i] = x.a[k];
      b1.a[i] = x.a[16 + k];
      b2.a[i] = x.a[32 + k];
      b3.a[i] = x.a[48 + k];
    }
  }
  // rows 1..3 rotated by A1..A3 (row_ror), row 0 as is
  template <int A1, int A2, int A3>
  static U ror_rows(const U& x) {
    const int A[4] = {0, A1, A2, A3};
    U r;
    for (int i = 0; i < 64; i++) r.a[i] = x.a[(i & ~15) | ((i - A[i >> 4]) & 15)];
    return r;
  }
  // S = 4: the sum over the four rows on every row; S = 2: rows c and c ^ 2
  template <int S>
  static U64 sum_rows(const U64& x) {
    U64 r;
    for (int i = 0; i < 64; i++) {
      const int k = i & 15;
      r.a[i] = S == 4 ? x.a[k] + x.a[16 + k] + x.a[32 + k] + x.a[48 + k] : x.a[i] + x.a[i ^ 32];
    }
    return r;
  }
  static uint64_t ballot(const B& b) {
    uint64_t m = 0;
    for (int i = 0; i < 64; i++) m |= (uint64_t)b.a[i] << i;
    return m;
  }
  // this lane's 16-bit limb of the 10-limb value at word off[lane] of row
  static U niels_limb(const uint32_t* row, const U& off) {
    U r;
    for (int i = 0; i < 64; i++) {
      cmtv::fe f;
      for (int j = 0; j < 10; j++) f.v[j] = row[off.a[i] + j];
      uint32_t b[8];
      cmtv::fe_tobytes(b, f);
      const int k = i & 15;
      r.a[i] = (b[k >> 1] >> (16 * (k & 1))) & 0xFFFF;
    }
    return r;
  }
  static U load_const(const uint16_t* tab, const U& k) {
    U r;
    for (int i = 0; i < 64; i++) r.a[i] = tab[k.a[i]];
    return r;
  }
};

// the LDS table policy: [tbl][neg][entry] one u32 per lane
struct HostRowTab {
  U t[2][2][9];
  void store(int tb, int neg, int e, const U& c) { t[tb][neg][e] = c; }
  U load(int tb, int neg, int e) const { return t[tb][neg][e]; }
};

}  // namespace hostlv

using namespace cmtv;
using hostlv::HostRow;

static void to_words(uint32_t* w, const uint8_t* b, int nw) {
  for (int i = 0; i < nw; i++)
    w[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
}

// ---- "mul": the field layer against a big-int reference -------------------------
typedef unsigned __int128 u128;
static const uint64_t P64[4] = {0xFFFFFFFFFFFFFFEDull, ~0ull, ~0ull, 0x7FFFFFFFFFFFFFFFull};
static void big_from_limbs(uint64_t r[4], const uint32_t* l) {
  uint64_t acc[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < 16; k++) {
    const int bit = 16 * k, w = bit / 64, sh = bit % 64;
    u128 v = (u128)l[k] << sh;
    for (int i = w; i < 5 && v; i++) {
      u128 s = (u128)acc[i] + (uint64_t)v;
      acc[i] = (uint64_t)s;
      v = (v >> 64) + (s >> 64);
    }
  }
  for (int it = 0; it < 3; it++) {
    u128 c = (u128)acc[4] * 38;
    acc[4] = 0;
    for (int i = 0; i < 5 && c; i++) {
      u128 s = (u128)acc[i] + (uint64_t)c;
      acc[i] = (uint64_t)s;
      c = (c >> 64) + (s >> 64);
    }
  }
  for (int it = 0; it < 4; it++) {
    bool ge = true;
    for (int i = 3; i >= 0; i--)
      if (acc[i] != P64[i]) {
        ge = acc[i] > P64[i];
        break;
      }
    if (!ge) break;
    u128 b = 0;
    for (int i = 0; i < 4; i++) {
      u128 d = (u128)acc[i] - P64[i] - (uint64_t)b;
      acc[i] = (uint64_t)d;
      b = (d >> 64) ? 1 : 0;
    }
  }
  for (int i = 0; i < 4; i++) r[i] = acc[i];
}
static void big_mul(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      u128 s = (u128)a[i] * b[j] + t[i + j] + (uint64_t)c;
      t[i + j] = (uint64_t)s;
      c = s >> 64;
    }
    t[i + 4] = (uint64_t)c;
  }
  uint64_t lo[4];
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)t[i + 4] * 38 + t[i] + (uint64_t)c;
    lo[i] = (uint64_t)s;
    c = s >> 64;
  }
  uint32_t l[16];
  for (int k = 0; k < 16; k++) l[k] = (uint32_t)(lo[k / 4] >> (16 * (k % 4))) & 0xFFFF;
  l[0] += (uint32_t)c * 38;
  big_from_limbs(r, l);
}

static int mul_selftest() {
  std::mt19937_64 rng(7);
  const RowCtx<HostRow> x(HostRow::lane());
  int bad = 0;
  for (int trial = 0; trial < 200; trial++) {
    hostlv::U f, g;
    // limbs up to the stated input bound 2^19.37 on some trials
    const uint32_t lim = trial % 3 == 0 ? 677000u : (trial % 3 == 1 ? 0x10000u : 0x10600u);
    for (int i = 0; i < 64; i++) {
      f.a[i] = (uint32_t)(rng() % lim);
      g.a[i] = (uint32_t)(rng() % lim);
    }
    hostlv::U h = trial & 1 ? rf_mul(x, f, g) : rf_sq(x, f);
    for (int row = 0; row < 4; row++) {
      uint64_t a[4], b[4], want[4], got[4];
      big_from_limbs(a, &f.a[16 * row]);
      big_from_limbs(b, &(trial & 1 ? g : f).a[16 * row]);
      big_mul(want, a, b);
      big_from_limbs(got, &h.a[16 * row]);
      for (int i = 0; i < 4; i++) bad += want[i] != got[i];
      for (int k = 0; k < 16; k++)
        if (h.a[16 * row + k] > 0x10000u + 128u) {
          fprintf(stderr, "limb %u above the carried bound\n", h.a[16 * row + k]);
          bad++;
        }
      // canonical test of h and of h - h
      const RowCanon<HostRow> cz = rf_canon<HostRow>(rf_sub(x, h, h));
      const RowCanon<HostRow> ch = rf_canon<HostRow>(h);
      const bool hz = (want[0] | want[1] | want[2] | want[3]) == 0;
      if (!cz.zero.a[16 * row] || ch.zero.a[16 * row] != hz || ch.odd.a[16 * row] != (bool)(want[0] & 1)) bad++;
    }
  }
  // values equal to p, 2p and 2^256 - 1 (non-canonical inputs of rf_canon)
  const uint64_t specials[3][4] = {{P64[0], P64[1], P64[2], P64[3]},
                                   {0xFFFFFFFFFFFFFFDAull, ~0ull, ~0ull, ~0ull},
                                   {~0ull, ~0ull, ~0ull, ~0ull}};
  for (int s = 0; s < 3; s++) {
    hostlv::U f;
    for (int i = 0; i < 64; i++) f.a[i] = (uint32_t)(specials[s][(i & 15) / 4] >> (16 * (i & 3))) & 0xFFFF;
    const RowCanon<HostRow> c = rf_canon<HostRow>(f);
    const bool want_zero = s < 2, want_odd = s == 2;  // 2^256 - 1 = 2p + 37
    if (c.zero.a[0] != want_zero || c.odd.a[0] != want_odd) bad++;
  }
  printf(bad ? "MISMATCH %d\n" : "ok\n", bad);
  return bad ? 1 : 0;
}

// comb of P (negated when neg), as the runtime's k_comb_build produces it
struct HostScratch {
  fe q[COMB_WINDOWS];
  void store(int j, const fe& v) { q[j] = v; }
  void load(int j, fe& v) const { v = q[j]; }
};
static std::vector<uint32_t> host_comb(const uint32_t pkw[8], bool neg, bool* ok) {
  std::vector<uint32_t> tab(COMB_TABLE_WORDS);
  ge_p3 A, nA;
  *ok = p3_frombytes(A, pkw);
  cached_neg_point(nA, A);
  for (int d = 1; d <= COMB_ENTRIES; d++) {
    HostScratch sc;
    comb_build_column(tab.data(), neg ? nA : A, d, sc);
  }
  return tab;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "mul")) return mul_selftest();
  // argv[1] == "row2": the two-wave form (r_part for R, then for A, r_join)
  const bool row2 = argc > 1 && !strcmp(argv[1], "row2");
  // argv[1] == "row4": the four-wave form (the high parts of A and R, the lo
  // wave's low windows of both, r_join4)
  const bool row4 = argc > 1 && !strcmp(argv[1], "row4");
  // argv[1] == "krow": registered keys (the keyed row kernel's path: the key's
  // radix-256 comb, the B table's radix-2^16 comb, -R decoded, r_keyed_join)
  const bool krow = argc > 1 && !strcmp(argv[1], "krow");
  std::map<std::string, std::pair<bool, std::vector<uint32_t>>> combs;
  LazyBTab bt;
  uint32_t n;
  if (fread(&n, 4, 1, stdin) != 1) return 1;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t mode = 0, pk[32], sig[64];
    uint32_t mlen;
    if (fread(&mode, 1, 1, stdin) != 1 || fread(pk, 32, 1, stdin) != 1 || fread(sig, 64, 1, stdin) != 1 ||
        fread(&mlen, 4, 1, stdin) != 1)
      return 1;
    std::vector<uint8_t> msg(mlen + 1);
    if (mlen && fread(msg.data(), mlen, 1, stdin) != 1) return 1;
    uint32_t pkw[8], sigw[16];
    to_words(pkw, pk, 8);
    to_words(sigw, sig, 16);
    SigPrep hp;
    if (mode)
      q_prepare<MODE_ZIP215>(hp, pkw, sigw, msg.data(), mlen, false);
    else
      q_prepare<MODE_GO_STDLIB>(hp, pkw, sigw, msg.data(), mlen, false);
    ge_p3 Bp;
    q_bcomb16(Bp, hp.u, bt);
    uint32_t bb[32];
    bpoint_store_bytes(bb, Bp);
    // this lane's 16-bit limb: row c & 1 = 0: A, 1: R
    hostlv::U limb, blimb;
    for (int l = 0; l < 64; l++) {
      const int c = l >> 4, k = l & 15;
      const uint8_t* src = (c & 1) ? sig : pk;
      limb.a[l] = src[2 * k] | (src[2 * k + 1] << 8);
      blimb.a[l] = (bb[8 * c + k / 2] >> (16 * (k & 1))) & 0xFFFF;
    }
    hostlv::HostRowTab tab;
    auto get_prep = [&](SigPrep& p) { p = hp; };
    auto get_b = [&]() { return blimb; };
    bool v;
    if (krow) {
      auto it = combs.find(std::string((const char*)pk, 32));
      if (it == combs.end()) {
        bool o;
        auto tab = host_comb(pkw, true, &o);
        it = combs.emplace(std::string((const char*)pk, 32), std::make_pair(o, std::move(tab))).first;
      }
      const RowCtx<HostRow> x(HostRow::lane());
      hostlv::U lr;
      for (int l = 0; l < 64; l++) lr.a[l] = sig[2 * (l & 15)] | (sig[2 * (l & 15) + 1] << 8);
      uint32_t tk[8], sw[8];
      q_keyed_challenge(tk, pkw, sigw, msg.data(), mlen);
      for (int j = 0; j < 8; j++) sw[j] = sigw[8 + j];
      const bool s_ok = (sw[7] & 0xE0000000u) == 0 && sc_is_canonical(sw);
      bool r_ok;
      const hostlv::U nr = mode ? r_decode_neg_r<MODE_ZIP215>(x, lr, sigw, r_ok)
                                : r_decode_neg_r<MODE_GO_STDLIB>(x, lr, sigw, r_ok);
      const hostlv::U d2 = x.cst(RowConst::d2);
      const uint32_t* kt = it->second.second.data();
      // as the kernel splits them: positions 15..0 on the A wave, 31..16 after [s]B on the B wave
      auto krow = [&](int j, int e) { return kt + ((size_t)j * COMB_ENTRIES + e) * COMB_ROW_WORDS; };
      hostlv::U va = rp_identity(x);
      uint32_t tk2[8];
      for (int j = 0; j < 8; j++) tk2[j] = tk[j];
      r_kcomb(x, va, tk, krow, 15, 0);
      hostlv::U vb = r_bcomb16(x, sw, [&](int e) { return bt.row(e); });
      r_kcomb(x, vb, tk2, krow, 31, 16);
      const hostlv::U ca = rp_to_cached(x, va, d2);
      const hostlv::U cb = rp_to_cached(x, vb, d2);
      const bool ok = it->second.first && s_ok && r_ok;
      v = mode ? r_keyed_join<MODE_ZIP215>(x, nr, ca, cb, ok) : r_keyed_join<MODE_GO_STDLIB>(x, nr, ca, cb, ok);
    } else if (row4) {
      const RowCtx<HostRow> x(HostRow::lane());
      hostlv::U la, lr;
      for (int l = 0; l < 64; l++) {
        const int k = l & 15;
        la.a[l] = pk[2 * k] | (pk[2 * k + 1] << 8);
        lr.a[l] = sig[2 * k] | (sig[2 * k + 1] << 8);
      }
      hostlv::HostRowTab ta, tr, tl;
      SigPrep p;
      bool a_dec, a_x0, r_dec, r_x0, a_ok, r_ok, r_canon;
      const hostlv::U d2 = x.cst(RowConst::d2);
      const hostlv::U ca = rp_to_cached(
          x, r_part<0, kRowLoWindows>(x, la, (pk[31] >> 7) != 0, ta, get_prep, p, a_dec, a_x0), d2);
      const hostlv::U cr = rp_to_cached(
          x, r_part<1, kRowLoWindows>(x, lr, (sig[31] >> 7) != 0, tr, get_prep, p, r_dec, r_x0), d2);
      const hostlv::U vl = r_sum_ar(x, limb, pkw, sigw, tl, get_prep, kRowLoWindows, p, a_ok, r_ok, r_canon);
      const bool ok = (p.flags & 4u) != 0 && a_ok && r_ok;
      v = mode ? r_join4<MODE_ZIP215>(x, vl, ca, cr, blimb, ok, r_canon)
               : r_join4<MODE_GO_STDLIB>(x, vl, ca, cr, blimb, ok, r_canon);
    } else if (row2) {
      const RowCtx<HostRow> x(HostRow::lane());
      hostlv::U la, lr;
      for (int l = 0; l < 64; l++) {
        const int k = l & 15;
        la.a[l] = pk[2 * k] | (pk[2 * k + 1] << 8);
        lr.a[l] = sig[2 * k] | (sig[2 * k + 1] << 8);
      }
      hostlv::HostRowTab ta, tr;
      SigPrep p;
      bool a_dec, a_x0, r_dec, r_x0;
      const hostlv::U vr = r_part<1>(x, lr, (sig[31] >> 7) != 0, tr, get_prep, p, r_dec, r_x0);
      const hostlv::U cr = rp_to_cached(x, vr, x.cst(RowConst::d2));
      const hostlv::U va = r_part<0>(x, la, (pk[31] >> 7) != 0, ta, get_prep, p, a_dec, a_x0);
      const bool ok = (p.flags & 4u) != 0 && a_dec && r_dec;
      const bool r_canon = y_is_canonical(sigw) && !(r_x0 && (sig[31] >> 7));
      v = mode ? r_join<MODE_ZIP215>(x, va, cr, blimb, ok, r_canon) : r_join<MODE_GO_STDLIB>(x, va, cr, blimb, ok, r_canon);
    } else {
      v = mode ? r_verify_split<MODE_ZIP215>(HostRow(), limb, pkw, sigw, tab, get_prep, get_b)
               : r_verify_split<MODE_GO_STDLIB>(HostRow(), limb, pkw, sigw, tab, get_prep, get_b);
    }
    const uint8_t o = v;
    fwrite(&o, 1, 1, stdout);
  }
  return 0;
}
