"""GPU parity on the half-size-scalar window schedules beyond the common 34
(tests/golden/wide_vectors.json: 35- and 36-window pairs, checked on the CPU
in tests/test_wide_vectors.py), and on the 64-window wide fallback, which no
searchable k reaches (forced with the CMTV_FORCE_WIDE knob).

The quad-family kernels (k_verify_quad_hs, k_verify_sr25519_quad_hs, the oct
and row forms) pick the window count per WAVE (the largest its 16 signatures need), and the radix-256 B digits
ride on the low windows whatever the count (quad.h q_straus_half). Each
vector is therefore placed inside a wave of ordinary signatures (honest and
bit-flipped), at a different lane position per wave, and the whole batch is
compared with the C oracle bit for bit, in both Ed25519 modes. The lane
kernels and the registered-key kernels (keyed.h / keyed_quad.h, which do not
split k) run the same batches.
Reference semantics: crypto/ed25519/ed25519.go:148-155 (Go 1.19 Verify) and
crypto/sr25519/pubkey.go:34-60.
"""
import json
import os

import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, pack_messages
from conftest import ED_FORMS, FORMS

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(kind):
    with open(os.path.join(ROOT, "tests", "golden", "wide_vectors.json")) as f:
        vs = json.load(f)[kind]
    return ([np.frombuffer(bytes.fromhex(v["pk"]), np.uint8) for v in vs],
            [np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vs],
            [bytes.fromhex(v["msg"]) for v in vs], vs)


def _mixed_batch(kind, waves_per_vector=1, seed=3):
    """Each wide vector in its own 16-signature wave, at lane position
    (3 + 5 w) % 16, the other 15 ordinary (20% with a flipped bit); then one
    wave holding every wide vector; then the wide vectors alone."""
    wpk, wsig, wmsg, _ = _load(kind)
    nw = len(wpk)
    n_fill = 16 * nw
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 256, (40, 32), dtype=np.uint8)
    kidx = rng.integers(0, 40, n_fill).astype(np.uint32)
    msgs = [rng.integers(0, 256, 116, dtype=np.uint8).tobytes() for _ in range(n_fill)]
    m, off = coracle.pack_msgs(msgs)
    if kind == "ed25519":
        fsig = coracle.sign_batch(keys, m, off, key_idx=kidx, nthreads=8)
        fpk = coracle.pubkeys_from_seeds(keys)[kidx]
    else:
        fsig = coracle.sr25519_sign_batch(keys, m, off, key_idx=kidx)
        fpk = coracle.sr25519_pubkeys(keys)[kidx]
    fsig = fsig.copy()
    for i in np.nonzero(rng.random(n_fill) < 0.2)[0]:
        fsig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
    pk, sig, mm = [], [], []
    for w in range(nw):
        pos = (3 + 5 * w) % 16
        for j in range(16):
            if j == pos:
                pk.append(wpk[w]); sig.append(wsig[w]); mm.append(wmsg[w])
            else:
                i = 16 * w + j
                pk.append(fpk[i]); sig.append(fsig[i]); mm.append(msgs[i])
    pk += wpk; sig += wsig; mm += wmsg          # a wave (or two) of wide ones
    pk += wpk[:1]; sig += wsig[:1]; mm += wmsg[:1]  # ragged tail
    m2, off2 = pack_messages(mm)
    return np.array(pk), np.array(sig), m2, off2


@pytest.mark.parametrize("kernel", ED_FORMS)
@pytest.mark.parametrize("mode", [MODE_GO_STDLIB, MODE_ZIP215])
def test_ed25519_wide_in_mixed_waves(form_ctx, kernel, mode):
    ctx = form_ctx(kernel)
    pk, sig, m, off = _mixed_batch("ed25519")
    exp = coracle.verify_batch(pk, sig, m, off, mode, nthreads=8)
    got, words = ctx.verify(pk, sig, m, off, mode, bitmap=True)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, bad[:20]
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: len(exp)]
    assert np.array_equal(bits, exp)
    # the committed verdicts, wherever the vectors sit
    _, _, _, vs = _load("ed25519")
    key = "go" if mode == MODE_GO_STDLIB else "zip215"
    alone = ctx.verify(pk[-len(vs) - 1:-1], sig[-len(vs) - 1:-1], *pack_messages(
        [bytes.fromhex(v["msg"]) for v in vs]), mode)
    assert [int(x) for x in alone] == [v[key] for v in vs]


@pytest.mark.parametrize("kernel", ["krow", "kquad", "lane"])
@pytest.mark.parametrize("mode", [MODE_GO_STDLIB, MODE_ZIP215])
def test_ed25519_wide_keyed(form_ctx, kernel, mode):
    ctx = form_ctx(kernel)
    pk, sig, m, off = _mixed_batch("ed25519", seed=4)
    uniq, idx = np.unique(pk, axis=0, return_inverse=True)
    ks = ctx.register_keys(uniq)
    exp = coracle.verify_batch(pk, sig, m, off, mode, nthreads=8)
    got = ctx.verify_indexed(ks, idx.astype(np.uint32).reshape(-1), sig, m, off, mode)
    ks.free()
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:20]


@pytest.mark.parametrize("kernel", ["quad", "lane"])
def test_sr25519_wide_in_mixed_waves(form_ctx, kernel):
    ctx = form_ctx(kernel)
    pk, sig, m, off = _mixed_batch("sr25519", seed=5)
    exp = coracle.sr25519_verify_batch(pk, sig, m, off, nthreads=8)
    got = ctx.verify_sr25519(pk, sig, m, off)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:20]
    _, _, _, vs = _load("sr25519")
    assert [int(x) for x in got[-len(vs) - 1:-1]] == [v["valid"] for v in vs]


def test_reference_keygen_vector_on_device(gpu_ctx):
    """privval/msgs_test.go:62,85: the device keygen of
    GenPrivKeyFromSecret("it's a secret") gives the reference's public key,
    and a device signature under it verifies (and a flipped one does not)."""
    from oracle import ed25519_ref as E

    with open(os.path.join(ROOT, "tests", "golden", "keygen_kat.json")) as f:
        v = json.load(f)["vectors"][0]
    seed = np.frombuffer(E.gen_priv_key_from_secret(v["secret"].encode()), np.uint8).reshape(1, 32)
    pk = gpu_ctx.pubkeys(seed)
    assert pk[0].tobytes().hex() == v["pubkey"]
    m, off = pack_messages([b"it's a message", b"another"])
    sig = gpu_ctx.sign(seed, m, off, key_idx=np.zeros(2, np.uint32))
    sig[1, 7] ^= 2
    got = gpu_ctx.verify(np.repeat(pk, 2, axis=0), sig, m, off, MODE_GO_STDLIB)
    assert list(got) == [1, 0]


@pytest.fixture(scope="module")
def forced_wide_ctxs():
    from conftest import _env_ctx

    return {k: _env_ctx(CMTV_FORCE_WIDE=1, CMTV_FORM=FORMS[k]) for k in ("row4", "row", "oct2", "quad")}


@pytest.mark.parametrize("kernel", ["row4", "row", "oct2", "quad"])
@pytest.mark.parametrize("mode,key", [(MODE_GO_STDLIB, "go"), (MODE_ZIP215, "zip215")])
def test_forced_wide_schedule_on_corpus(forced_wide_ctxs, corpus, mode, key, kernel):
    """CMTV_FORCE_WIDE: every quad (or oct) takes the wide fallback (k1 = k,
    k2 = 1, 64 windows, B digits on windows 0..32): the edge-case corpus and
    mixed batches stay bit-exact."""
    ctx = forced_wide_ctxs[kernel]
    msg, off = pack_messages(corpus["msgs"])
    got = ctx.verify(corpus["pk"], corpus["sig"], msg, off, mode)
    assert np.array_equal(got, corpus[key]), np.nonzero(got != corpus[key])[0][:10]
    pk, sig, m, off = _mixed_batch("ed25519", seed=6)
    exp = coracle.verify_batch(pk, sig, m, off, mode, nthreads=8)
    assert np.array_equal(ctx.verify(pk, sig, m, off, mode), exp)


def test_forced_wide_schedule_sr25519(forced_wide_ctxs):
    forced_wide_ctx = forced_wide_ctxs["quad"]
    pk, sig, m, off = _mixed_batch("sr25519", seed=7)
    exp = coracle.sr25519_verify_batch(pk, sig, m, off, nthreads=8)
    assert np.array_equal(forced_wide_ctx.verify_sr25519(pk, sig, m, off), exp)
    with open(os.path.join(ROOT, "tests", "golden", "sr25519_corpus.json")) as f:
        vecs = json.load(f)["vectors"]
    cpk = np.array([np.frombuffer(bytes.fromhex(v["pk"]), np.uint8) for v in vecs])
    csig = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vecs])
    cm, coff = pack_messages([bytes.fromhex(v["msg"]) for v in vecs])
    assert [int(x) for x in forced_wide_ctx.verify_sr25519(cpk, csig, cm, coff)] == [v["valid"] for v in vecs]
