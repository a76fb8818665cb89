// Host emulation of the 4-lane quad kernel (cometbft_amd/csrc/quad.h): four
// std::threads run the same source in lockstep and exchange DPP quad_perm
// operands through a barrier. Test infrastructure only.
//   stdin/stdout protocol as hostcheck.cpp (verify mode only).
#define CMTV_HD inline
#define CMTV_BOUNDS_CHECK 1
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#include "../../cometbft_amd/csrc/oct.h"
#include "../../cometbft_amd/csrc/quad.h"
#include "../../cometbft_amd/csrc/sr25519_quad.h"
#include "../../cometbft_amd/csrc/keyed_quad.h"
#include "lazy_btab.h"
#include <map>
#include <string>

using namespace cmtv;

// sense-reversing spin barrier for the 4 lane threads (a futex barrier makes
// the ~10^5 exchanges per signature dominate the run time)
struct SpinBarrier {
  int n = 4;
  std::atomic<int> count{0};
  std::atomic<int> gen{0};
  void arrive_and_wait() {
    const int g = gen.load(std::memory_order_acquire);
    if (count.fetch_add(1, std::memory_order_acq_rel) == n - 1) {
      count.store(0, std::memory_order_relaxed);
      gen.store(g + 1, std::memory_order_release);
      return;
    }
    for (int spins = 0; gen.load(std::memory_order_acquire) == g; spins++)
      if (spins > 256) std::this_thread::yield();
  }
};

struct Exchange {
  SpinBarrier bar;
  fe slot[8];
};

struct HostQuad {
  int ln;
  Exchange* ex;
  int lane() const { return ln; }
  template <int PAT>
  void perm(fe& o, const fe& v) const {
    ex->slot[ln] = v;
    ex->bar.arrive_and_wait();
    const fe r = ex->slot[(PAT >> (2 * ln)) & 3];
    ex->bar.arrive_and_wait();
    o = r;
  }
  template <int PAT>
  void add_perm(fe& o, const fe& src, const fe& b) const {
    fe t;
    perm<PAT>(t, src);
    for (int i = 0; i < 10; i++) o.v[i] = t.v[i] + b.v[i];
  }
  template <int PAT>
  void xor_perm(fe& o, const fe& src, uint32_t k) const {
    perm<PAT>(o, src);
    for (int i = 0; i < 10; i++) o.v[i] ^= k;
  }
  template <int PAT>
  void perm_lane3(fe& o, const fe& src) const {
    perm<PAT>(o, src);
    for (int i = 0; i < 10; i++) o.v[i] = lane() == 3 ? o.v[i] : 0u;
  }
  template <int PAT>
  void permc(fe& o, const fe& v) const {
    perm<PAT>(o, v);
  }
  template <int PAT>
  uint32_t perm32(uint32_t x) const {
    fe t, o;
    fe_0(t);
    t.v[0] = x;
    perm<PAT>(o, t);
    return o.v[0];
  }
  bool any(bool x) const { return x; }  // the four lanes of one quad agree
};

// the oct policy (oct.h): 8 threads, quad_perm inside each half, and the
// upper quad's words reaching the lower one (DPP row_shl:4)
struct HostOct {
  int ln;
  Exchange* ex;
  int lane() const { return ln & 3; }
  bool upper() const { return (ln & 4) != 0; }
  template <int PAT>
  void perm(fe& o, const fe& v) const {
    ex->slot[ln] = v;
    ex->bar.arrive_and_wait();
    const fe r = ex->slot[(ln & 4) + ((PAT >> (2 * (ln & 3))) & 3)];
    ex->bar.arrive_and_wait();
    o = r;
  }
  template <int PAT>
  void add_perm(fe& o, const fe& src, const fe& b) const {
    fe t;
    perm<PAT>(t, src);
    for (int i = 0; i < 10; i++) o.v[i] = t.v[i] + b.v[i];
  }
  template <int PAT>
  void xor_perm(fe& o, const fe& src, uint32_t k) const {
    perm<PAT>(o, src);
    for (int i = 0; i < 10; i++) o.v[i] ^= k;
  }
  template <int PAT>
  void perm_lane3(fe& o, const fe& src) const {
    perm<PAT>(o, src);
    for (int i = 0; i < 10; i++) o.v[i] = lane() == 3 ? o.v[i] : 0u;
  }
  template <int PAT>
  void permc(fe& o, const fe& v) const {
    perm<PAT>(o, v);
  }
  template <int PAT>
  uint32_t perm32(uint32_t x) const {
    fe t, o;
    fe_0(t);
    t.v[0] = x;
    perm<PAT>(o, t);
    return o.v[0];
  }
  void from_upper(fe& o, const fe& v) const {
    ex->slot[ln] = v;
    ex->bar.arrive_and_wait();
    const fe r = ex->slot[ln < 4 ? ln + 4 : ln];
    ex->bar.arrive_and_wait();
    o = r;
  }
  uint32_t from_upper32(uint32_t x) const {
    fe t, o;
    fe_0(t);
    t.v[0] = x;
    from_upper(o, t);
    return o.v[0];
  }
  // W is the max over the signature's lanes: both quads compute the same pair
  bool any(bool x) const { return x; }
};

using HostBTab = LazyBTab;  // lazy_btab.h: rows computed on first use

struct HostScratch {
  fe q[COMB_WINDOWS];
  void store(int j, const fe& v) { q[j] = v; }
  void load(int j, fe& v) const { v = q[j]; }
};

// comb of P (negated when neg), as the runtime's k_comb_build produces it
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

int main(int argc, char** argv) {
  // argv[1] == "sr": sr25519 records { pk[32], sig[64], u32 mlen, msg } (no mode byte)
  // argv[1] == "sr2": the same through k_verify_sr25519_quad_split's path --
  // the merlin transcript and [u]B computed once as its helper wave does, the
  // tables built before the scalars arrive (q_tables_early: R's table is of
  // -R, a negative k2 flips R's digits at lookup), then q_verify_sr_split<true>
  const bool sr2 = argc > 1 && !strcmp(argv[1], "sr2");
  // argv[1] == "sr3": sr25519 through k_verify_sr25519_quad_hs's path (as
  // "quad3" below, q_verify_sr_hs)
  const bool sr3 = argc > 1 && !strcmp(argv[1], "sr3");
  const bool sr = sr2 || sr3 || (argc > 1 && !strcmp(argv[1], "sr"));
  // argv[1] == "keyed": Ed25519 records, verified through registered-key combs (keyed_quad.h)
  const bool keyed = argc > 1 && !strcmp(argv[1], "keyed");
  // argv[1] == "keyedmix": one lane, the key's radix-256 comb with B over the
  // B table's radix-2^16 comb (keyed.h keyed_comb_mixed, kCombMixed)
  const bool keyedmix = argc > 1 && !strcmp(argv[1], "keyedmix");
  // argv[1] == "keyed16": the keyed quad verifier with [s]B over the B
  // table's radix-2^16 comb (q_verify_keyed_split<MODE, true>, the keyed
  // split kernel's default)
  const bool keyed16 = argc > 1 && !strcmp(argv[1], "keyed16");
  // argv[1] == "oct": Ed25519 records through the 8-lane verifier (oct.h)
  const bool oct = argc > 1 && !strcmp(argv[1], "oct");
  // argv[1] == "quad2" / "oct2": the split kernels' path -- the scalars and
  // [u]B (q_prepare, q_bcomb16) computed once as the helper wave would, the
  // quad / oct verifier taking them through its callbacks
  const bool quad2 = argc > 1 && !strcmp(argv[1], "quad2");
  const bool oct2 = argc > 1 && !strcmp(argv[1], "oct2");
  // argv[1] == "quad3": k_verify_quad_hs's path (quad.h q_verify_hs) -- the
  // scalars, [u]B and every window's summed addend (h_window_addend over the
  // four lanes' tables) computed once as its helper wave would; the window
  // count is the signature's own raised by i % 3 (a workgroup's count can be
  // any other signature's), 64 when wide
  const bool quad3 = argc > 1 && !strcmp(argv[1], "quad3");
  std::vector<uint32_t> bcomb;
  std::map<std::string, std::pair<bool, std::vector<uint32_t>>> combs;
  if (keyed) {
    uint32_t bw[8];
    bool bok;
    basepoint_words(bw);
    bcomb = host_comb(bw, false, &bok);
  }
  uint32_t prog[SR_PREFIX_WORDS];  // the program the runtime uploads
  const int nops = sr_prefix_state(prog);
  if (nops <= 0) return 2;
  HostBTab bt;
  uint32_t n, k2_neg_count = 0;
  if (fread(&n, 4, 1, stdin) != 1) return 1;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t mode = 0, pk[32], sig[64];
    uint32_t mlen;
    if ((!sr && fread(&mode, 1, 1, stdin) != 1) || fread(pk, 32, 1, stdin) != 1 || fread(sig, 64, 1, stdin) != 1 ||
        fread(&mlen, 4, 1, stdin) != 1)
      return 1;
    std::vector<uint8_t> buf(mlen + 16, 0xEE);
    uint8_t* mp = buf.data() + 4 + (i % 4);
    if (mlen && fread(mp, mlen, 1, stdin) != 1) return 1;
    uint32_t pkw[8], sigw[16];
    to_words(pkw, pk, 8);
    to_words(sigw, sig, 16);
    bool kok = false;
    const uint32_t* kt = nullptr;
    if (keyed || keyedmix || keyed16) {
      auto it = combs.find(std::string((const char*)pk, 32));
      if (it == combs.end()) {
        bool o;
        auto tab = host_comb(pkw, true, &o);
        it = combs.emplace(std::string((const char*)pk, 32), std::make_pair(o, std::move(tab))).first;
      }
      kok = it->second.first;
      kt = it->second.second.data();
    }
    if (keyedmix) {
      ge_p3 acc;
      const bool ok = keyed_comb_mixed<CombWindow>(acc, pkw, kok, sigw, mp, mlen, kt, bt);
      uint8_t o = (mode ? check_R<MODE_ZIP215>(acc, sigw) : check_R<MODE_GO_STDLIB>(acc, sigw)) && ok;
      fwrite(&o, 1, 1, stdout);
      continue;
    }
    Exchange ex;
    bool res[8];
    std::vector<std::thread> th;
    SigPrep hp;
    uint32_t bpt[40];
    if (sr2 || sr3) {
      ArrayStrobeState st;
      sr_prepare(hp, pkw, sigw, mp, mlen, prog, nops, st, false);
      ge_p3 Bp;
      q_bcomb16(Bp, hp.u, bt);
      bpoint_store(bpt, Bp);
      k2_neg_count += (hp.flags & 1u) ? 1 : 0;
    }
    if (quad2 || oct2 || quad3) {
      if (mode)
        q_prepare<MODE_ZIP215>(hp, pkw, sigw, mp, mlen, false);
      else
        q_prepare<MODE_GO_STDLIB>(hp, pkw, sigw, mp, mlen, false);
      ge_p3 Bp;
      q_bcomb16(Bp, hp.u, bt);
      bpoint_store(bpt, Bp);
    }
    auto get_prep = [&](SigPrep& p) { p = hp; };
    if (sr2) {
      for (int l = 0; l < 4; l++)
        th.emplace_back([&, l] {
          HostQuad q{l, &ex};
          QArrayTab ta, tr;
          auto get_b = [&](fe& c) {
            for (int j = 0; j < 10; j++) c.v[j] = bpt[10 * l + j];
          };
          res[l] = q_verify_sr_split<true>(q, pkw, sigw, bt, ta, tr, get_prep, get_b);
        });
    }
    if (quad2 || oct2) {
      ex.bar.n = oct2 ? 8 : 4;
      for (int l = 0; l < (oct2 ? 8 : 4); l++)
        th.emplace_back([&, l] {
          QArrayTab ta, tr;
          auto get_b = [&](fe& c) {
            for (int j = 0; j < 10; j++) c.v[j] = bpt[10 * (l & 3) + j];
          };
          if (oct2) {
            HostOct q{l, &ex};
            res[l] = mode ? o_verify_split<MODE_ZIP215, true>(q, pkw, sigw, bt, ta, get_prep, get_b)
                          : o_verify_split<MODE_GO_STDLIB, true>(q, pkw, sigw, bt, ta, get_prep, get_b);
          } else {
            HostQuad q{l, &ex};
            res[l] = mode ? q_verify_split<MODE_ZIP215, true>(q, pkw, sigw, bt, ta, tr, get_prep, get_b)
                          : q_verify_split<MODE_GO_STDLIB, true>(q, pkw, sigw, bt, ta, tr, get_prep, get_b);
          }
        });
    }
    if (quad3 || sr3) {
      const bool wide = (hp.flags & 2u) != 0;
      const int own = (int)((hp.flags >> 8) & 0xFFu);
      const int W = wide ? HS_WIDE_WINDOWS : (own + (int)(i % 3) > HS_MAX_WINDOWS ? HS_MAX_WINDOWS : own + (int)(i % 3));
      hp.flags |= (uint32_t)W << 16;
      QArrayTab ta[4], tr[4];
      fe S[4];
      uint32_t tA[8], tR[8];
      hs_digits16(tA, hp.k1, W);
      hs_digits16(tR, hp.k2, W);
      sc_shift_out(tA, 4);
      sc_shift_out(tR, 4);
      // the helper's part of [u]B: the top `pre` comb positions (0..16, by i)
      const int pre = (int)(i % 17);
      BComb16 bc;
      bc.init(hp.u);
      for (int k = 0; k < pre; k++) bc.step(bt);
      uint32_t bpt3[40];
      bpoint_store(bpt3, bc.P);
      for (int l = 0; l < 4; l++)
        th.emplace_back([&, l] {
          HostQuad q{l, &ex};
          auto get_s = [&](int win, fe& c) {
            ex.bar.arrive_and_wait();  // every lane's tables are built
            if (l == 0) {
              const int dA = (int)sc_shift_out(tA, 4) - 8;
              const int dR = (int)sc_shift_out(tR, 4) - 8;
              auto rd = [&](int P, int e, int cc, fe& r) { r = (P == 0 ? ta[cc] : tr[cc]).t[e]; };
              h_window_addend(S, rd, dA, dR, (hp.flags & 1u) != 0);
            }
            ex.bar.arrive_and_wait();
            c = S[l];
            (void)win;
          };
          auto get_b = [&](fe& c) {
            for (int j = 0; j < 10; j++) c.v[j] = bpt3[10 * l + j];
          };
          if (sr3)
            res[l] = q_verify_sr_hs(q, pkw, sigw, bt, ta[l], tr[l], 16 - pre, get_prep, get_s, get_b);
          else
            res[l] = mode ? q_verify_hs<MODE_ZIP215>(q, pkw, sigw, bt, ta[l], tr[l], 16 - pre, get_prep, get_s, get_b)
                          : q_verify_hs<MODE_GO_STDLIB>(q, pkw, sigw, bt, ta[l], tr[l], 16 - pre, get_prep, get_s, get_b);
        });
    }
    if (oct) {
      ex.bar.n = 8;
      for (int l = 0; l < 8; l++)
        th.emplace_back([&, l] {
          HostOct q{l, &ex};
          QArrayTab ta;
          res[l] = mode ? o_verify<MODE_ZIP215>(q, pkw, sigw, mp, mlen, bt, ta)
                        : o_verify<MODE_GO_STDLIB>(q, pkw, sigw, mp, mlen, bt, ta);
        });
    }
    for (int l = 0; l < (oct || quad2 || oct2 || sr2 || quad3 || sr3 ? 0 : 4); l++)
      th.emplace_back([&, l] {
        HostQuad q{l, &ex};
        QArrayTab ta, tr;
        ArrayStrobeState st;
        if (sr)
          res[l] = q_verify_sr(q, pkw, sigw, mp, mlen, prog, nops, st, bt, ta, tr);
        else if (keyed)
          res[l] = mode ? q_verify_keyed<MODE_ZIP215>(q, pkw, kok, sigw, mp, mlen, kt, bcomb.data())
                        : q_verify_keyed<MODE_GO_STDLIB>(q, pkw, kok, sigw, mp, mlen, kt, bcomb.data());
        else if (keyed16) {
          auto get_k = [&](uint32_t tk[8]) { q_keyed_challenge(tk, pkw, sigw, mp, mlen); };
          auto get_r = [&](fe& rc, bool& r_ok) {
            ge_p3 R;
            r_ok = mode ? q_keyed_decode_r<MODE_ZIP215>(R, sigw) : q_keyed_decode_r<MODE_GO_STDLIB>(R, sigw);
            fe one;
            fe_1(one);
            fe_pick(rc, l, R.X, R.Y, one, R.T);
          };
          res[l] = mode ? q_verify_keyed_split<MODE_ZIP215, true>(q, kok, sigw, kt, nullptr, get_k, get_r, bt)
                        : q_verify_keyed_split<MODE_GO_STDLIB, true>(q, kok, sigw, kt, nullptr, get_k, get_r, bt);
        }
        else
          res[l] = mode ? q_verify<MODE_ZIP215>(q, pkw, sigw, mp, mlen, bt, ta, tr)
                        : q_verify<MODE_GO_STDLIB>(q, pkw, sigw, mp, mlen, bt, ta, tr);
      });
    for (auto& t : th) t.join();
    if (res[0] != res[1] || res[0] != res[2] || res[0] != res[3]) {
      fprintf(stderr, "lanes disagree on vector %u\n", i);
      return 2;
    }
    uint8_t o = res[0];
    fwrite(&o, 1, 1, stdout);
  }
  // sr2: how many signatures took the negative-k2 (flipped R digit) path
  if (sr2) fprintf(stderr, "k2_neg %u of %u\n", k2_neg_count, n);
  return 0;
}
