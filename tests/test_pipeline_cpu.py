"""CPU check of the cross-height pipeline's host logic (tests/host/pipecheck.cpp).

cometbft_amd/csrc/commit.cpp and pipeline.cpp are compiled unchanged, with
AddressSanitizer + UBSan, against tests/host/fake_runtime.cpp -- a stand-in
for the device half of the library whose "device" reads each chunk's pinned
staging the way the kernels do (templated sign-bytes rebuilt with
signbytes.h and checked against the host's offsets) and verifies with the C
restatement of Go 1.19 ed25519.Verify (oracle/cmtv_oracle.c), lazily, when
the chunk is waited for. A 240-commit chain with assorted faults over four
validator sets (one with a 31-byte key) goes through the reference loops
written out from types/validator_set.go:667-826, the one-batch path and the
pipeline in eight configurations (chunks of 7 to 1000 signatures, 2-4
slots, 1-8 threads, 1-3 devices, registered keys, a device failing mid-call,
a device retired by another call while a chunk is in flight on it);
every commit's outcome must agree."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cometbft_amd", "csrc")
HOST = os.path.join(ROOT, "tests", "host")
BIN = os.path.join(HOST, "pipecheck")
SRCS = [os.path.join(HOST, "pipecheck.cpp"), os.path.join(HOST, "fake_runtime.cpp"),
        os.path.join(CSRC, "commit.cpp"), os.path.join(CSRC, "pipeline.cpp")]
FLAGS = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
         "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]


def _build(san="address,undefined", binary=BIN):
    deps = SRCS + [os.path.join(ROOT, "oracle", "cmtv_oracle.c"), os.path.join(ROOT, "include", "cmtverify.h")] + \
        [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if os.path.exists(binary) and os.path.getmtime(binary) >= max(os.path.getmtime(d) for d in deps):
        return binary
    objdir = os.path.join(ROOT, "build", "pipecheck_" + san.replace(",", "_"))
    os.makedirs(objdir, exist_ok=True)
    flags = [f for f in FLAGS if not f.startswith("-fsanitize")] + [f"-fsanitize={san}"]
    objs = []
    procs = []
    for src in SRCS:
        o = os.path.join(objdir, os.path.basename(src) + ".o")
        procs.append(subprocess.Popen(["g++"] + flags + ["-c", src, "-o", o]))
        objs.append(o)
    o = os.path.join(objdir, "cmtv_oracle.o")
    procs.append(subprocess.Popen(["gcc", "-O2", "-g", f"-fsanitize={san}", "-c",
                                   os.path.join(ROOT, "oracle", "cmtv_oracle.c"), "-o", o]))
    objs.append(o)
    for p in procs:
        assert p.wait() == 0, "pipecheck build failed"
    tmp = f"{binary}.{os.getpid()}"
    subprocess.run(["g++", f"-fsanitize={san}", "-o", tmp] + objs + ["-lpthread"], check=True)
    os.replace(tmp, binary)
    return binary


def test_pipeline_host_logic_matches_reference_loops():
    try:
        b = _build()
    except (OSError, subprocess.CalledProcessError, AssertionError) as e:
        pytest.fail(f"could not build pipecheck: {e}")
    r = subprocess.run([b, "240"], capture_output=True, text=True, timeout=600,
                       env={**os.environ, "ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1",
                            "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "pipecheck ok (64 runs)" in r.stdout
    assert "single: 240 commits x 3 kinds x 2, 0 mismatches" in r.stdout
    for kind in (0, 1, 2):
        assert f"kind {kind} mode 0: 240 commits" in r.stdout


def test_pipeline_concurrent_callers_under_tsan():
    """ThreadSanitizer (the reference's `go test -race`, tests.mk:67-70;
    SURVEY 5): the same host code built with -fsanitize=thread, one context
    shared by a pipelined cmtv_verify_commits caller (direct and packed
    chunks on two fake devices, the host worker pool), a single-commit
    cmtv_verify_commit caller and a thread allocating / freeing pinned blocks;
    every outcome checked against the reference loops, any race report fails
    (halt_on_error)."""
    try:
        b = _build("thread", os.path.join(HOST, "pipecheck_tsan"))
    except (OSError, subprocess.CalledProcessError, AssertionError) as e:
        pytest.fail(f"could not build pipecheck_tsan: {e}")
    r = subprocess.run([b, "120", "race"], capture_output=True, text=True, timeout=900,
                       env={**os.environ, "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "race: 6 iterations, 0 mismatches" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr
