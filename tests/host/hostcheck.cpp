// Host-side build of the device math (cometbft_amd/csrc/verify_core.h) with
// operand-bound assertions on (CMTV_BOUNDS_CHECK). Test infrastructure only:
// lets the per-lane pipeline be checked against the oracle without a GPU.
//   input  (stdin):  u32 n, then n x { u8 mode, u8 pk[32], u8 sig[64], u32 mlen, u8 msg[mlen] }
//   output (stdout): n bytes of verdicts
//   argv[1] == "sign": n x { u8 seed[32], u32 mlen, msg } -> n x { pk[32], sig[64] }
//   argv[1] == "half":  verify input as above, through verify_one_half (the
//                       lane kernel's half-size-scalar pipeline)
//   argv[1] == "keyed": verify input as above, through registered-key combs
//                       (keyed.h; one comb per distinct pk)
//   argv[1] == "zipc":  as "keyed", with ZIP-215's final check by coset
//                       (verify_core.h check_R_zip_coset) instead of decoding R
//   argv[1] == "coset": n x { u8 rp[32], u8 r[32] } -> n verdicts of the coset
//                       check for R' = decode(rp) against R bytes r
#define CMTV_HD inline
#define CMTV_BOUNDS_CHECK 1
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>
#include "../../cometbft_amd/csrc/keyed.h"

using namespace cmtv;

struct HostBTab {
  std::vector<uint32_t> rows;
  HostBTab() : rows(2 * BTAB_ENTRIES * BTAB_ROW_WORDS) {
    for (int e = 0; e < 2 * BTAB_ENTRIES; e++) btab_entry(&rows[e * BTAB_ROW_WORDS], e % BTAB_ENTRIES + 1, e >= BTAB_ENTRIES);
  }
  void load_fe(int e, int c, fe& r) const {
    const uint32_t* p = &rows[e * BTAB_ROW_WORDS + c * BTAB_COORD_WORDS];
    for (int i = 0; i < 10; i++) r.v[i] = p[i];
  }
};

struct HostATab {
  ge_cached t[8];
  void load_fe(int e, int c, fe& r) const {
    r = c == 0 ? t[e].YpX : c == 1 ? t[e].YmX : c == 2 ? t[e].Z : t[e].T2d;
  }
  void store(int e, const ge_cached& r) { t[e] = r; }
};

struct HostScratch {
  fe q[COMB_WINDOWS];
  void store(int j, const fe& v) { q[j] = v; }
  void load(int j, fe& v) const { v = q[j]; }
};

// comb of P (negated when neg) as the runtime's k_comb_build produces it
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

static void to_words(uint32_t* w, const uint8_t* b, int nw) {
  for (int i = 0; i < nw; i++) w[i] = b[4 * i] | (b[4 * i + 1] << 8) | (b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
}
static void from_words(uint8_t* b, const uint32_t* w, int nw) {
  for (int i = 0; i < nw; i++)
    for (int j = 0; j < 4; j++) b[4 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

int main(int argc, char** argv) {
  HostBTab bt;
  uint32_t n;
  if (fread(&n, 4, 1, stdin) != 1) return 1;
  const bool sign = argc > 1 && !strcmp(argv[1], "sign");
  const bool keyed = argc > 1 && !strcmp(argv[1], "keyed");
  const bool half = argc > 1 && !strcmp(argv[1], "half");
  const bool zipc = argc > 1 && !strcmp(argv[1], "zipc");
  const bool coset = argc > 1 && !strcmp(argv[1], "coset");
  std::vector<uint32_t> bcomb;
  std::map<std::string, std::pair<bool, std::vector<uint32_t>>> combs;
  if (keyed || zipc) {
    uint32_t bw[8];
    bool bok;
    basepoint_words(bw);
    bcomb = host_comb(bw, false, &bok);
  }
  for (uint32_t i = 0; i < n; i++) {
    if (sign) {
      uint8_t seed[32];
      uint32_t mlen;
      if (fread(seed, 32, 1, stdin) != 1 || fread(&mlen, 4, 1, stdin) != 1) return 1;
      std::vector<uint8_t> msg(mlen + 1);
      if (mlen && fread(msg.data(), mlen, 1, stdin) != 1) return 1;
      uint32_t sw[8], pk[8], sig[16];
      to_words(sw, seed, 8);
      pubkey_from_seed(pk, sw, bt);
      sign_one(sig, sw, msg.data(), mlen, bt);
      uint8_t out[96];
      from_words(out, pk, 8);
      from_words(out + 32, sig, 16);
      fwrite(out, 96, 1, stdout);
      continue;
    }
    if (coset) {
      uint8_t rp[32], r[32];
      if (fread(rp, 32, 1, stdin) != 1 || fread(r, 32, 1, stdin) != 1) return 1;
      uint32_t rpw[8], rw[8];
      to_words(rpw, rp, 8);
      to_words(rw, r, 8);
      ge_p3 Rp;
      const bool ok = p3_frombytes(Rp, rpw);
      uint8_t o = ok && check_R_zip_coset(Rp, rw);
      fwrite(&o, 1, 1, stdout);
      continue;
    }
    uint8_t mode, pk[32], sig[64];
    uint32_t mlen;
    if (fread(&mode, 1, 1, stdin) != 1 || fread(pk, 32, 1, stdin) != 1 || fread(sig, 64, 1, stdin) != 1 ||
        fread(&mlen, 4, 1, stdin) != 1)
      return 1;
    // place the message at a varying misalignment (the device reads aligned words)
    std::vector<uint8_t> buf(mlen + 16, 0xEE);
    uint8_t* mp = buf.data() + 4 + (i % 4);
    if (mlen && fread(mp, mlen, 1, stdin) != 1) return 1;
    uint32_t pkw[8], sigw[16];
    to_words(pkw, pk, 8);
    to_words(sigw, sig, 16);
    if (keyed || zipc) {
      auto it = combs.find(std::string((const char*)pk, 32));
      if (it == combs.end()) {
        bool kok;
        auto tab = host_comb(pkw, true, &kok);
        it = combs.emplace(std::string((const char*)pk, 32), std::make_pair(kok, std::move(tab))).first;
      }
      const bool kok = it->second.first;
      const uint32_t* kt = it->second.second.data();
      bool v;
      if (zipc && mode) {
        ge_p3 acc;
        const bool ok = keyed_comb<CombWindow>(acc, pkw, kok, sigw, mp, mlen, kt, bcomb.data());
        v = check_R_zip_coset(acc, sigw) && ok;
      } else {
        v = mode ? verify_keyed<MODE_ZIP215, CombWindow>(pkw, kok, sigw, mp, mlen, kt, bcomb.data())
                 : verify_keyed<MODE_GO_STDLIB, CombWindow>(pkw, kok, sigw, mp, mlen, kt, bcomb.data());
      }
      uint8_t o = v;
      fwrite(&o, 1, 1, stdout);
      continue;
    }
    HostATab at, ar;
    bool v;
    if (half)
      v = mode ? verify_one_half<MODE_ZIP215>(pkw, sigw, mp, mlen, at, ar, bt)
               : verify_one_half<MODE_GO_STDLIB>(pkw, sigw, mp, mlen, at, ar, bt);
    else
      v = mode ? verify_one<MODE_ZIP215>(pkw, sigw, mp, mlen, at, bt)
               : verify_one<MODE_GO_STDLIB>(pkw, sigw, mp, mlen, at, bt);
    uint8_t o = v;
    fwrite(&o, 1, 1, stdout);
  }
  return 0;
}
