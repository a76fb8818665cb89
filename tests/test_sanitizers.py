"""Host-side AddressSanitizer + UBSan (the reference runs
`go test -race`, tests.mk:67-70; this is the native-code counterpart).

 * tests/host/abicheck_san: runtime.cpp + commit.cpp built with host-only
   -fsanitize=address,undefined (cometbft_amd/csrc/Makefile `san`), linked
   with the same gfx950 kernel objects, driven through the C ABI only.
   Without a GPU it checks the ENODEV path and the device-free entry points;
   on the GPU (marked gpu) it verifies corpus vectors in both modes through
   the single-device, sharded ([0, 0, 0]), BatchVerifier, verdict-cache and
   registered-key paths with 4 concurrent callers on one context.
 * the host builds of the device math (tests/host/hostcheck.cpp,
   halfcheck.cpp, shardcheck.cpp) under -fsanitize=address,undefined.
Any sanitizer report fails the test (halt_on_error)."""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN_BIN = os.path.join(ROOT, "tests", "host", "abicheck_san")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def _vectors(corpus, path, n=300):
    idx = list(range(0, len(corpus["msgs"]), max(1, len(corpus["msgs"]) // n)))[:n]
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(idx)))
        for i in idx:
            m = corpus["msgs"][i]
            f.write(corpus["pk"][i].tobytes() + corpus["sig"][i].tobytes() + struct.pack("<I", len(m)) + m)
            f.write(bytes([int(corpus["go"][i]), int(corpus["zip215"][i])]))
    return len(idx)


TSAN_BIN = os.path.join(ROOT, "tests", "host", "abicheck_tsan")
# the HIP runtime is not instrumented: its own threads' accesses are ignored
TSAN_ENV = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:ignore_noninstrumented_modules=1:report_signal_unsafe=0")


def _abicheck(tmp_path, corpus, binary=SAN_BIN, target="san", env=ENV):
    if not os.path.exists(binary):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "cometbft_amd", "csrc"), target], check=True)
    vec = str(tmp_path / "vectors.bin")
    _vectors(corpus, vec)
    return subprocess.run([binary, vec, "4"], capture_output=True, text=True, env=env, timeout=600)


def test_runtime_under_asan_ubsan_without_device(tmp_path, corpus):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: see the gpu variant")
    r = _abicheck(tmp_path, corpus)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "no device" in r.stdout and "0 failures" in r.stdout


@pytest.mark.gpu
def test_runtime_under_asan_ubsan_on_device(tmp_path, corpus):
    r = _abicheck(tmp_path, corpus)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout and "no device" not in r.stdout


def test_runtime_under_tsan_without_device(tmp_path, corpus):
    """ThreadSanitizer build of runtime.cpp + commit.cpp + pipeline.cpp
    (Makefile `tsan`, host code only): the device-free entry points."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: see the gpu variant")
    r = _abicheck(tmp_path, corpus, TSAN_BIN, "tsan", TSAN_ENV)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "no device" in r.stdout and "0 failures" in r.stdout


@pytest.mark.gpu
def test_runtime_under_tsan_on_device(tmp_path, corpus):
    """The same under ThreadSanitizer on the GPU: 4 concurrent host-batch
    callers on one context, then a pipelined cmtv_verify_commits caller
    (direct and packed chunks), a single-commit cmtv_verify_commit caller and
    a host-batch caller sharing one context (abicheck commit_concurrency);
    any race report in the library's host code fails."""
    r = _abicheck(tmp_path, corpus, TSAN_BIN, "tsan", TSAN_ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "0 failures" in r.stdout and "no device" not in r.stdout
    assert "ThreadSanitizer" not in r.stderr


def _san_build(src, out, flags):
    out = os.path.join(ROOT, "build", out)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["g++", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined"] + flags +
                   ["-o", out, src], check=True)
    return out


def test_device_math_host_builds_under_asan_ubsan(corpus):
    host = os.path.join(ROOT, "tests", "host")
    hc = _san_build(os.path.join(host, "hostcheck.cpp"), "hostcheck_san", ["-std=c++17"])
    idx = list(range(0, len(corpus["msgs"]), 23))
    buf = [struct.pack("<I", len(idx))]
    for i in idx:
        m = corpus["msgs"][i]
        buf.append(bytes([0]) + corpus["pk"][i].tobytes() + corpus["sig"][i].tobytes() + struct.pack("<I", len(m)) + m)
    for arg in (None, "half"):
        out = subprocess.run([hc] + ([arg] if arg else []), input=b"".join(buf), capture_output=True, env=ENV,
                             timeout=900)
        assert out.returncode == 0, out.stderr[-3000:]
        assert np.array_equal(np.frombuffer(out.stdout, np.uint8), corpus["go"][idx])
    half = _san_build(os.path.join(host, "halfcheck.cpp"), "halfcheck_san", ["-std=c++17"])
    rng = np.random.default_rng(5)
    L = 2**252 + 27742317777372353535851937790883648493
    ks = [0, 1, L - 1] + [int.from_bytes(rng.bytes(32), "little") % L for _ in range(500)]
    r = subprocess.run([half], input=struct.pack("<I", len(ks)) + b"".join(k.to_bytes(32, "little") for k in ks),
                       capture_output=True, env=ENV, timeout=300)
    assert r.returncode == 0 and len(r.stdout) == 130 * len(ks), r.stderr[-2000:]
    sh = _san_build(os.path.join(host, "shardcheck.cpp"), "shardcheck_san", ["-std=c++17"])
    r = subprocess.run([sh], input=b"".join(struct.pack("<3Q", n, g, 64) for n in (0, 1, 65, 10**6) for g in (1, 8)),
                       capture_output=True, env=ENV, timeout=60)
    assert r.returncode == 0 and len(r.stdout) == 8 * 24, r.stderr
