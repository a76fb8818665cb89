"""The device math (cometbft_amd/csrc/*.h) compiled for the host with operand
bound assertions on (tests/host/hostcheck.cpp), run over the golden corpus:
the generic pipeline (verify_core.h verify_one) and the registered-key comb
pipeline (keyed.h verify_keyed) must reproduce both committed verdict vectors
bit for bit. No GPU needed; the GPU kernels are the same source."""
import os
import struct
import subprocess

import numpy as np
import pytest

from tests.host import hostbuild

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "host", "hostcheck.cpp")
BIN = os.path.join(ROOT, "build", "hostcheck")
QSRC = os.path.join(ROOT, "tests", "host", "quadcheck.cpp")
QBIN = os.path.join(ROOT, "build", "quadcheck")


@pytest.fixture(scope="module")
def hostcheck():
    return _build(SRC, BIN, ["-std=c++17"])


@pytest.fixture(scope="module")
def quadcheck():
    return _build(QSRC, QBIN, ["-std=c++20", "-pthread"])


def _build(src, binary, flags):
    return hostbuild.build(src, binary, flags)


def _run(binary, arg, corpus, idx, mode):
    buf = [struct.pack("<I", len(idx))]
    for i in idx:
        m = corpus["msgs"][i]
        buf.append(bytes([mode]) + corpus["pk"][i].tobytes() + corpus["sig"][i].tobytes() + struct.pack("<I", len(m)) + m)
    args = [binary] + ([arg] if arg else [])
    out = subprocess.run(args, input=b"".join(buf), capture_output=True, check=True, timeout=600).stdout
    return np.frombuffer(out, np.uint8)


@pytest.mark.parametrize("mode", [0, 1])
def test_half_scalar_lane_pipeline_matches_corpus(hostcheck, corpus, mode):
    """verify_one_half (the lane kernel: half-size scalars, 33+ windows, R
    table, X = [k2](R' - R)) over the whole corpus at every misalignment."""
    idx = list(range(len(corpus["msgs"])))
    got = _run(hostcheck, "half", corpus, idx, mode)
    want = corpus["go"] if mode == 0 else corpus["zip215"]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), corpus["cats"][int(i)]) for i in bad[:10]]


@pytest.mark.parametrize("mode", [0, 1])
def test_generic_pipeline_matches_corpus(hostcheck, corpus, mode):
    idx = list(range(len(corpus["msgs"])))
    got = _run(hostcheck, None, corpus, idx, mode)
    want = corpus["go"] if mode == 0 else corpus["zip215"]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), corpus["cats"][i]) for i in bad[:10]]


def _keyed_subset(corpus):
    # every non-honest vector plus a slice of the honest ones; the comb
    # build is ~10 ms per distinct key on the host
    cats = corpus["cats"]
    idx = [i for i, c in enumerate(cats) if c not in ("honest", "random")]
    idx += [i for i, c in enumerate(cats) if c in ("honest", "random")][:64]
    return sorted(idx)


@pytest.mark.parametrize("mode", [0, 1])
def test_keyed_pipeline_matches_corpus(hostcheck, corpus, mode):
    idx = _keyed_subset(corpus)
    got = _run(hostcheck, "keyed", corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


def test_zip_coset_check_matches_corpus(hostcheck, corpus):
    """ZIP-215's final check by coset (verify_core.h zip_coset: R' + E[8]
    against y_R and R's sign bit, no square root) on the keyed pipeline."""
    idx = _keyed_subset(corpus)
    got = _run(hostcheck, "zipc", corpus, idx, 1)
    want = corpus["zip215"][idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


def test_zip_coset_check_fuzz(hostcheck):
    """The coset check against decode-R-and-[8](R' - R) (the oracle) for R' =
    [s]B, [s]B + a torsion point and pure torsion points, and R = every
    translate R' + T (T in E[8]) with the sign bit as encoded and flipped and
    the y >= p encoding where one exists, plus random R bytes."""
    import random

    from oracle import ed25519_ref as E

    P, L = E.P, E.L
    t8, y = None, 2
    while t8 is None:  # a point of order 8: [L] of a curve point with full torsion
        x = E._recover_x(y, 0)
        if x is not None:
            q = E.scalar_mult(L, (x, y, 1, x * y % P))
            r, k = q, 1
            while not E.is_identity(r) and k < 9:
                r, k = E.point_add(r, q), k + 1
            if k == 8:
                t8 = q
        y += 1
    e8 = [E.IDENTITY]
    for _ in range(7):
        e8.append(E.point_add(e8[-1], t8))

    def ref(rp, rb):
        R = E.decode_point(rb)
        if R is None:
            return 0
        d = E.point_add(rp, E.point_neg(R))
        for _ in range(3):
            d = E.point_double(d)
        return int(E.is_identity(d))

    rnd = random.Random(11)
    cases = []
    for trial in range(24):
        rp = E.scalar_mult(rnd.randrange(L), E.B)
        if trial % 3 == 1:
            rp = E.point_add(rp, e8[rnd.randrange(1, 8)])
        if trial % 8 == 2:
            rp = e8[rnd.randrange(8)]
        rpb = E.encode_point(rp)
        rp = E.decode_point(rpb)  # the point the host check decodes
        for t in e8:
            enc = E.encode_point(E.point_add(rp, t))
            for flip in (0, 1):
                b = bytearray(enc)
                b[31] ^= 0x80 * flip
                cases.append((rpb, bytes(b)))
                v = int.from_bytes(bytes(b), "little")
                y_, sgn = v & ((1 << 255) - 1), v >> 255
                if y_ + P < (1 << 255):
                    cases.append((rpb, ((y_ + P) | (sgn << 255)).to_bytes(32, "little")))
        for _ in range(4):
            cases.append((rpb, rnd.getrandbits(256).to_bytes(32, "little")))
    buf = [struct.pack("<I", len(cases))] + [a + b for a, b in cases]
    out = subprocess.run([hostcheck, "coset"], input=b"".join(buf), capture_output=True, check=True,
                         timeout=600).stdout
    got = np.frombuffer(out, np.uint8)
    want = np.array([ref(E.decode_point(a), b) for a, b in cases], np.uint8)
    assert 0 < want.sum() < len(cases)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]


@pytest.mark.parametrize("mode", [0, 1])
def test_oct_pipeline_matches_corpus(quadcheck, corpus, mode):
    """The 8-lane oct kernel's source (oct.h): eight host threads in lockstep,
    the two quads' Straus chains merged by the row-shift exchange."""
    idx = _keyed_subset(corpus)[1::6]
    got = _run(quadcheck, "oct", corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


@pytest.mark.parametrize("kind", ["quad2", "oct2", "quad3"])
@pytest.mark.parametrize("mode", [0, 1])
def test_split_pipelines_match_corpus(quadcheck, corpus, mode, kind):
    """The helper-wave kernels' path: scalars and [u]B (the 16-position
    radix-2^16 comb, q_bcomb16) computed once per signature as the helper
    wave does, the quad / oct verifier taking them through its callbacks
    (no fixed-base digits in its windows)."""
    idx = _keyed_subset(corpus)[2::7]
    got = _run(quadcheck, kind, corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


@pytest.mark.parametrize("mode", [0, 1])
def test_keyed_mixed_comb_matches_corpus(quadcheck, corpus, mode):
    """kCombMixed (keyed.h keyed_comb_mixed): [k](-A) over the key's
    radix-256 comb, [s]B over the B table's radix-2^16 comb -- the lane path
    for key sets without wide combs -- on the corpus, both modes."""
    idx = _keyed_subset(corpus)
    got = _run(quadcheck, "keyedmix", corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


@pytest.mark.parametrize("mode", [0, 1])
def test_keyed_quad_b16_matches_corpus(quadcheck, corpus, mode):
    """The keyed quad split kernel's [s]B over the B table's radix-2^16 comb
    (q_verify_keyed_split<MODE, true>) in 4-thread lockstep, both modes."""
    idx = _keyed_subset(corpus)[::3]
    got = _run(quadcheck, "keyed16", corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


@pytest.mark.parametrize("mode", [0, 1])
def test_quad_pipeline_matches_corpus(quadcheck, corpus, mode):
    """The 4-lane quad kernel's source (quad.h), four host threads in lockstep
    standing in for the DPP quad_perm exchanges (every adversarial vector and
    a slice of the honest ones: the lockstep emulation is ~40 ms a vector)."""
    idx = _keyed_subset(corpus)[::3]
    got = _run(quadcheck, None, corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


HSRC = os.path.join(ROOT, "tests", "host", "halfcheck.cpp")
HBIN = os.path.join(ROOT, "build", "halfcheck")
L = 2**252 + 27742317777372353535851937790883648493


@pytest.mark.parametrize("parity", ["odd", "any"])
def test_half_scalar_decomposition(parity):
    """halfscalar.h (the device source, host-compiled): k1 == k2 k (mod 8L),
    0 <= k1, |k2| < 2^(4W - 2) for the pair's window count W (33..37) unless
    flagged wide (then k1 = k, k2 = 1, W = 64), L not dividing k2. "odd"
    (GO_STDLIB): k2 odd; W > 33 for ~1.2% of k, W > 34 ~5e-5, wide rarer.
    "any" (ZIP215): the shorter reduced basis vector, always inside 33
    windows. The Lehmer schedule must give exactly the pair of the
    one-step-per-round Euclid."""
    binary = _build(HSRC, HBIN, ["-std=c++17"])
    rng = np.random.default_rng(215)
    ks = [0, 1, 2, 3, L - 1, L - 2, 2**127, 2**128 - 1, 2**134, 2**252]
    ks += [int.from_bytes(rng.bytes(32), "little") % L for _ in range(20000)]
    buf = struct.pack("<I", len(ks)) + b"".join(k.to_bytes(32, "little") for k in ks)
    out = subprocess.run([binary, parity], input=buf, capture_output=True, check=True, timeout=120).stdout
    assert len(out) == 130 * len(ks)
    wide = 0
    windows = {}
    for j, k in enumerate(ks):
        rec = out[130 * j: 130 * j + 65]
        assert rec == out[130 * j + 65: 130 * (j + 1)], j  # Lehmer == exact steps
        k1 = int.from_bytes(rec[:32], "little")
        k2 = int.from_bytes(rec[32:64], "little")
        f = rec[64]
        w = (f >> 2) + 32
        if f & 2:
            wide += 1
            assert (k1, k2, f & 1, w) == (k, 1, 0, 64), j
            continue
        assert 33 <= w <= 37, (j, w)
        windows[w] = windows.get(w, 0) + 1
        s2 = -k2 if f & 1 else k2
        if parity == "odd":
            assert k2 & 1, j
        assert 0 < k2 < L, j
        bound = 2 ** (4 * w - 2)
        assert k1 < bound and 0 < k2 < bound, j
        if w > 33:  # the smallest window count that holds the pair
            assert max(k1.bit_length(), k2.bit_length()) > 4 * (w - 1) - 2, j
        assert (k1 - s2 * k) % (8 * L) == 0, j
    assert wide <= 8, wide  # wide: the boundary k (0, 1, 2^252, ...)
    if parity == "any":
        assert set(windows) == {33}, windows
    else:
        assert 0.005 < windows.get(34, 0) / len(ks) < 0.03, windows  # ~1.2%
        assert sum(c for w, c in windows.items() if w > 34) <= 20, windows


@pytest.mark.parametrize("mode", [0, 1])
def test_keyed_quad_pipeline_matches_corpus(quadcheck, corpus, mode):
    """keyed_quad.h (registered-key combs, one signature per DPP quad; four
    host threads in lockstep) over the non-honest vectors and a slice of the
    honest ones."""
    idx = _keyed_subset(corpus)[::2]
    got = _run(quadcheck, "keyed", corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


RSRC = os.path.join(ROOT, "tests", "host", "rowcheck.cpp")
RBIN = os.path.join(ROOT, "build", "rowcheck")


@pytest.fixture(scope="module")
def rowcheck():
    return _build(RSRC, RBIN, ["-std=c++20"])


def test_row_field_layer(rowcheck):
    """row.h's radix-2^16 product (16 column terms per lane, three carry
    rounds), squaring and canonical zero / parity test against a big-int
    reference, at the stated input bound (2^19.37) and on p, 2p, 2^256 - 1."""
    out = subprocess.run([rowcheck, "mul"], capture_output=True, check=True, timeout=120).stdout
    assert out.strip() == b"ok"


@pytest.mark.parametrize("form", ["row", "row2", "row4"])
@pytest.mark.parametrize("mode", [0, 1])
def test_row_pipeline_matches_corpus(rowcheck, corpus, mode, form):
    """The one-signature-per-wave row kernel's source (row.h r_verify_split)
    on 64-lane arrays with its operand bounds asserted, the scalars and [u]B
    from the helper wave's code (q_prepare, q_bcomb16): every non-honest
    vector and a slice of the honest ones. row2: the two-wave form (r_part
    for R and for A, r_join); row4: the four-wave form (the high parts of A
    and R from [2^84]P, the low windows of both, r_join4)."""
    idx = _keyed_subset(corpus)
    got = _run(rowcheck, None if form == "row" else form, corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]


@pytest.mark.parametrize("mode", [0, 1])
def test_keyed_row_pipeline_matches_corpus(rowcheck, corpus, mode):
    """The keyed row kernel's source (row.h r_decode_neg_r, r_kcomb over the
    key's radix-256 comb built as k_comb_build does, r_bcomb16 over the B
    table's rows, r_keyed_join) on 64-lane arrays."""
    idx = _keyed_subset(corpus)
    got = _run(rowcheck, "krow", corpus, idx, mode)
    want = (corpus["go"] if mode == 0 else corpus["zip215"])[idx]
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(idx[int(i)], corpus["cats"][idx[int(i)]]) for i in bad[:10]]
