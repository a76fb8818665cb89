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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "host", "hostcheck.cpp")
BIN = os.path.join(ROOT, "build", "hostcheck")


@pytest.fixture(scope="module")
def hostcheck():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    deps = [SRC] + [os.path.join(ROOT, "cometbft_amd", "csrc", f) for f in os.listdir(os.path.join(ROOT, "cometbft_amd", "csrc")) if f.endswith(".h")]
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(d) for d in deps):
        subprocess.run(["g++", "-O2", "-std=c++17", "-o", BIN, SRC], check=True)
    return BIN


def _run(binary, arg, corpus, idx, mode):
    buf = [struct.pack("<I", len(idx))]
    for i in idx:
        m = corpus["msgs"][i]
        buf.append(bytes([mode]) + corpus["pk"][i].tobytes() + corpus["sig"][i].tobytes() + struct.pack("<I", len(m)) + m)
    args = [binary] + ([arg] if arg else [])
    out = subprocess.run(args, input=b"".join(buf), capture_output=True, check=True, timeout=600).stdout
    return np.frombuffer(out, np.uint8)


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
