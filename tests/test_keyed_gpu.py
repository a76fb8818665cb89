"""GPU parity of registered-key verification (keyed.h / keyed_quad.h comb paths,
cmtv_register_keys + cmtv_verify_ed25519_indexed[_device]): verdicts must equal
the corpus' committed verdicts and the C oracle's, bit for bit, both modes.
Kernels (conftest.py FORMS, forced with CMTV_FORM): "krow" the keyed row
kernel, "kquad" the keyed quad kernel with two helper waves, "lane" the lane
kernels over the radix-256 key combs with B's radix-2^16 comb (kCombMixed),
"wide" the lane kernels over radix-2^16 key combs
(cmtv_register_keys_ex(CMTV_KEYS_WIDE), rows staged by LDS-DMA)."""
import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, pack_messages
from cometbft_amd import _native as N

pytestmark = pytest.mark.gpu


KERNELS = ["krow", "kquad", "lane", "wide"]


def _ctx(kernel, request):
    return request.getfixturevalue("form_ctx")("lane" if kernel == "wide" else kernel)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("mode,key", [(MODE_GO_STDLIB, "go"), (MODE_ZIP215, "zip215")])
def test_corpus_bit_exact_keyed(request, corpus, mode, key, kernel):
    gpu_ctx = _ctx(kernel, request)
    pk = corpus["pk"]
    uniq, idx = np.unique(pk, axis=0, return_inverse=True)  # 748 keys: 47 GiB of wide combs
    ks = gpu_ctx.register_keys(uniq, wide=kernel == "wide")
    assert len(ks) == uniq.shape[0]
    msg, off = pack_messages(corpus["msgs"])
    valid, words = gpu_ctx.verify_indexed(ks, idx.astype(np.uint32).reshape(-1), corpus["sig"], msg, off, mode,
                                          bitmap=True)
    exp = corpus[key]
    bad = np.nonzero(valid != exp)[0]
    assert bad.size == 0, [(corpus["cats"][i], int(valid[i]), int(exp[i])) for i in bad[:20]]
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: len(exp)]
    assert np.array_equal(bits, exp)
    ks.free()


@pytest.mark.parametrize("wide", [False, True])
def test_corpus_through_the_batched_kernels(corpus, wide):
    """The whole corpus through k_verify_keyed_batch at KB = 8
    (CMTV_KEYED_BATCH_MIN_WAVES=1 batches any size): the coset check of
    ZIP-215 and the shared inversion of GO_STDLIB on every adversarial R
    (non-canonical, small and mixed order), s and key category."""
    from conftest import _env_ctx

    ctx = _env_ctx(CMTV_FORM="lane,klane", CMTV_KEYED_BATCH_MIN_WAVES=1)
    uniq, idx = np.unique(corpus["pk"], axis=0, return_inverse=True)
    ks = ctx.register_keys(uniq, wide=wide)
    msg, off = pack_messages(corpus["msgs"])
    for mode, key in ((MODE_GO_STDLIB, "go"), (MODE_ZIP215, "zip215")):
        valid, words = ctx.verify_indexed(ks, idx.astype(np.uint32).reshape(-1), corpus["sig"], msg, off, mode,
                                          bitmap=True)
        bad = np.nonzero(valid != corpus[key])[0]
        assert bad.size == 0, [(corpus["cats"][i], int(valid[i])) for i in bad[:20]]
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: len(valid)]
        assert np.array_equal(bits, corpus[key])
    ks.free()


def _valset_commits(n_keys, n_sigs, seed):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n_keys, 32), dtype=np.uint8)
    kidx = rng.integers(0, n_keys, n_sigs).astype(np.uint32)
    msgs = [rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes() for _ in range(n_sigs)]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sign_batch(seeds, m, off, key_idx=kidx, nthreads=8)
    pk = coracle.pubkeys_from_seeds(seeds)
    return pk, kidx, sig, m, off, rng


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("n", [1, 15, 16, 17, 63, 64, 65, 3000, 12289])
def test_keyed_matches_generic_and_oracle(request, n, kernel):
    gpu_ctx = _ctx(kernel, request)
    pk, kidx, sig, m, off, rng = _valset_commits(150, n, 7 + n)
    sig = sig.copy()
    for i in np.nonzero(rng.random(n) < 0.2)[0]:
        sig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
    ks = gpu_ctx.register_keys(pk, wide=kernel == "wide")
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk[kidx], sig, m, off, mode, nthreads=8)
        got, words = gpu_ctx.verify_indexed(ks, kidx, sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp)
        assert np.array_equal(gpu_ctx.verify(pk[kidx], sig, m, off, mode), exp)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        assert np.array_equal(bits[:n], exp) and not bits[n:].any()
    ks.free()


@pytest.mark.parametrize("wide", [False, True])
def test_undecodable_and_noncanonical_keys(gpu_ctx, gpu_ctx_lane, corpus, wide):
    # keys the corpus marks off-curve / non-canonical, each used by its own vectors
    sel = [i for i, c in enumerate(corpus["cats"]) if c in ("offcurve_A", "noncanonical_A", "small_order_A")]
    assert sel
    pk = corpus["pk"][sel]
    msgs = [corpus["msgs"][i] for i in sel]
    m, off = pack_messages(msgs)
    gpu_ctx = gpu_ctx_lane if wide else gpu_ctx
    ks = gpu_ctx.register_keys(pk, wide=wide)
    for mode, key in ((MODE_GO_STDLIB, "go"), (MODE_ZIP215, "zip215")):
        got = gpu_ctx.verify_indexed(ks, np.arange(len(sel), dtype=np.uint32), corpus["sig"][sel], m, off, mode)
        assert np.array_equal(got, corpus[key][sel])
    ks.free()


def test_out_of_range_index(gpu_ctx):
    import torch

    pk, kidx, sig, m, off, _ = _valset_commits(4, 70, 3)
    ks = gpu_ctx.register_keys(pk)
    bad = kidx.copy()
    bad[5] = 4
    with pytest.raises(N.CmtvError) as ei:
        gpu_ctx.verify_indexed(ks, bad, sig, m, off)
    assert ei.value.code == N.CMTV_EINVAL
    # device entry point: the out-of-range entry is invalid, the rest verify
    dev = torch.device("cuda:0")
    t_idx = torch.from_numpy(bad.view(np.int32)).to(dev)
    t_sig = torch.from_numpy(sig).to(dev)
    t_msg = torch.from_numpy(np.concatenate([m, np.zeros(16, np.uint8)])).to(dev)
    t_off = torch.from_numpy(off.view(np.int32)).to(dev)
    t_valid = torch.zeros(70, dtype=torch.uint8, device=dev)
    t_bm = torch.zeros(2, dtype=torch.int64, device=dev)
    gpu_ctx.verify_indexed_device(ks, 70, t_idx.data_ptr(), t_sig.data_ptr(), t_msg.data_ptr(), t_off.data_ptr(),
                                  MODE_GO_STDLIB, t_valid.data_ptr(), t_bm.data_ptr())
    torch.cuda.synchronize()
    got = t_valid.cpu().numpy()
    exp = np.ones(70, np.uint8)
    exp[5] = 0
    assert np.array_equal(got, exp)
    ks.free()


def test_keyset_belongs_to_its_context(gpu_ctx, gpu_ctx_lane):
    pk, kidx, sig, m, off, _ = _valset_commits(2, 3, 5)
    ks = gpu_ctx.register_keys(pk)
    with pytest.raises(N.CmtvError):
        gpu_ctx_lane.verify_indexed(ks, kidx, sig, m, off)
    ks.free()


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("n", [530_000, 1_100_003])
def test_keyed_batch_inversion(gpu_ctx_lane, corpus, n, wide):
    """k_verify_keyed_batch (configs[2]'s lane path): KB = 4 / 8 signatures
    per lane share one field inversion (Montgomery's trick) -- GO_STDLIB's
    encode of R', ZIP-215's coset check (verify_core.h zip_coset). n =
    530,000 runs the KB = 4 form; 1,100,003 one 2^20 chunk at KB = 8 plus a
    ragged 51,427-signature tail on the plain kernel. The key set mixes 150
    honest keys with the corpus' off-curve keys (their combs are garbage, Z
    may vanish: their signatures must fail without spoiling the lane's
    others) and non-canonical / small-order keys; 1% of the signatures carry
    a flipped bit. Verdicts must equal the oracle's and the unbatched
    kernel's (KB = 1: CMTV_KEYED_BATCH_MIN_WAVES above any launch) bit for
    bit; with wide, over the radix-2^16 combs (rows staged by LDS-DMA; same
    verdicts, ZIP-215 too)."""
    from conftest import _env_ctx

    rng = np.random.default_rng(n)
    seeds = rng.integers(0, 256, (150, 32), dtype=np.uint8)
    honest = coracle.pubkeys_from_seeds(seeds)
    cats = corpus["cats"]
    odd = [i for i, c in enumerate(cats) if c in ("offcurve_A", "noncanonical_A", "small_order_A")][:24]
    pk = np.concatenate([honest, corpus["pk"][odd]])
    n_h = honest.shape[0]
    kidx = (np.arange(n) % n_h).astype(np.uint32)
    # every 97th signature by one of the corpus keys (with that vector's sig and msg)
    spots = np.arange(5, n, 97)
    m1 = np.frombuffer(np.random.default_rng(1).bytes(116), np.uint8)
    m = np.tile(m1, n).reshape(n, 116)
    m[:, :8] = np.arange(n, dtype=np.uint64).view(np.uint8).reshape(n, 8)  # distinct messages
    m = m.reshape(-1)
    off = (np.arange(n + 1, dtype=np.uint64) * 116).astype(np.uint32)
    sig = coracle.sign_batch(seeds, m, off, key_idx=kidx, nthreads=16).copy()
    for j, sp in enumerate(spots[: 4 * len(odd)]):
        t = odd[j % len(odd)]
        kidx[sp] = n_h + (j % len(odd))
        sig[sp] = corpus["sig"][t]
    flips = rng.choice(n, n // 100, replace=False)
    sig[flips, rng.integers(0, 64, flips.size)] ^= (1 << rng.integers(0, 8, flips.size)).astype(np.uint8)
    exp = coracle.verify_batch(pk[kidx], sig, m, off, MODE_GO_STDLIB, nthreads=16)
    assert 0 < exp.sum() < n
    ks = gpu_ctx_lane.register_keys(pk, wide=wide)
    got = gpu_ctx_lane.verify_indexed(ks, kidx, sig, m, off, MODE_GO_STDLIB)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, (bad[:10], kidx[bad[:10]])
    # ZIP-215 through the same batches: the coset check (no decode of R)
    exp_z = coracle.verify_batch(pk[kidx], sig, m, off, MODE_ZIP215, nthreads=16)
    got_z = gpu_ctx_lane.verify_indexed(ks, kidx, sig, m, off, MODE_ZIP215)
    bad = np.nonzero(got_z != exp_z)[0]
    assert bad.size == 0, (bad[:10], kidx[bad[:10]])
    ks.free()
    plain = _env_ctx(CMTV_FORM="lane,klane", CMTV_KEYED_BATCH_MIN_WAVES=1 << 20)
    ks2 = plain.register_keys(pk, wide=wide)
    assert np.array_equal(plain.verify_indexed(ks2, kidx, sig, m, off, MODE_GO_STDLIB), got)
    assert np.array_equal(plain.verify_indexed(ks2, kidx, sig, m, off, MODE_ZIP215), got_z)
    ks2.free()
