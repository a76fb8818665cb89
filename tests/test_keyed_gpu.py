"""GPU parity of registered-key verification (keyed.h / keyed_quad.h comb paths,
cmtv_register_keys + cmtv_verify_ed25519_indexed[_device]): verdicts must equal
the corpus' committed verdicts and the C oracle's, bit for bit, both modes."""
import numpy as np
import pytest

from oracle import coracle
from cometbft_amd import MODE_GO_STDLIB, MODE_ZIP215, pack_messages
from cometbft_amd import _native as N

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel", ["quad2", "quad", "lane"])
@pytest.mark.parametrize("mode,key", [(MODE_GO_STDLIB, "go"), (MODE_ZIP215, "zip215")])
def test_corpus_bit_exact_keyed(gpu_ctx, gpu_ctx_quad1, gpu_ctx_lane, corpus, mode, key, kernel):
    gpu_ctx = {"quad2": gpu_ctx, "quad": gpu_ctx_quad1, "lane": gpu_ctx_lane}[kernel]
    pk = corpus["pk"]
    uniq, idx = np.unique(pk, axis=0, return_inverse=True)
    ks = gpu_ctx.register_keys(uniq)
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


def _valset_commits(n_keys, n_sigs, seed):
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n_keys, 32), dtype=np.uint8)
    kidx = rng.integers(0, n_keys, n_sigs).astype(np.uint32)
    msgs = [rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes() for _ in range(n_sigs)]
    m, off = coracle.pack_msgs(msgs)
    sig = coracle.sign_batch(seeds, m, off, key_idx=kidx, nthreads=8)
    pk = coracle.pubkeys_from_seeds(seeds)
    return pk, kidx, sig, m, off, rng


@pytest.mark.parametrize("kernel", ["quad2", "quad", "lane"])
@pytest.mark.parametrize("n", [1, 15, 16, 17, 63, 64, 65, 3000, 12289])
def test_keyed_matches_generic_and_oracle(gpu_ctx, gpu_ctx_quad1, gpu_ctx_lane, n, kernel):
    gpu_ctx = {"quad2": gpu_ctx, "quad": gpu_ctx_quad1, "lane": gpu_ctx_lane}[kernel]
    pk, kidx, sig, m, off, rng = _valset_commits(150, n, 7 + n)
    sig = sig.copy()
    for i in np.nonzero(rng.random(n) < 0.2)[0]:
        sig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
    ks = gpu_ctx.register_keys(pk)
    for mode in (MODE_GO_STDLIB, MODE_ZIP215):
        exp = coracle.verify_batch(pk[kidx], sig, m, off, mode, nthreads=8)
        got, words = gpu_ctx.verify_indexed(ks, kidx, sig, m, off, mode, bitmap=True)
        assert np.array_equal(got, exp)
        assert np.array_equal(gpu_ctx.verify(pk[kidx], sig, m, off, mode), exp)
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        assert np.array_equal(bits[:n], exp) and not bits[n:].any()
    ks.free()


def test_undecodable_and_noncanonical_keys(gpu_ctx, corpus):
    # keys the corpus marks off-curve / non-canonical, each used by its own vectors
    sel = [i for i, c in enumerate(corpus["cats"]) if c in ("offcurve_A", "noncanonical_A", "small_order_A")]
    assert sel
    pk = corpus["pk"][sel]
    msgs = [corpus["msgs"][i] for i in sel]
    m, off = pack_messages(msgs)
    ks = gpu_ctx.register_keys(pk)
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
