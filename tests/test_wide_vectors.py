"""CPU checks of tests/golden/wide_vectors.json (made by
tests/golden/make_wide.py): signatures whose challenge k needs more than the
common 34 windows of the half-size-scalar split (halfscalar.h): 35, 36 and
37-window pairs, which random data reaches for only ~5e-5, ~3e-6 and ~3e-7
of k.

 - the stored verdicts are re-derived by both oracles (Python big-int
   restatements and oracle/liboracle.so), both Ed25519 modes and sr25519;
 - every vector's k takes the recorded window count in the host build of
   halfscalar.h;
 - the host builds of the device pipelines (hostcheck "half" = lane
   half-scalar Straus, quadcheck = the 4-lane quad kernel source) reproduce
   the verdicts through that schedule.
The same vectors run on the GPU in tests/test_wide_gpu.py."""
import json
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import coracle
from oracle import ed25519_ref as E
from oracle import sr25519_ref as S

from test_host_math import HBIN, HSRC, QBIN, QSRC, SRC, BIN, _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def wide():
    with open(os.path.join(ROOT, "tests", "golden", "wide_vectors.json")) as f:
        doc = json.load(f)
    def arr(vs):
        return {"pk": np.array([np.frombuffer(bytes.fromhex(v["pk"]), np.uint8) for v in vs]),
                "sig": np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vs]),
                "msgs": [bytes.fromhex(v["msg"]) for v in vs], "cats": [v["cat"] for v in vs], "raw": vs}
    return arr(doc["ed25519"]), arr(doc["sr25519"])


def _windows(ks):
    binary = _build(HSRC, HBIN, ["-std=c++17"])
    buf = struct.pack("<I", len(ks)) + b"".join(k.to_bytes(32, "little") for k in ks)
    out = subprocess.run([binary], input=buf, capture_output=True, check=True).stdout
    return [(out[130 * j + 64] >> 2) + 32 for j in range(len(ks))]


def test_ed25519_wide_verdicts_and_flags(wide):
    ed, _ = wide
    assert {"honest", "s_flip", "mixed_R", "mixed_A"} <= set(ed["cats"])
    ks = []
    for v in ed["raw"]:
        pk, sig, m = (bytes.fromhex(v[k]) for k in ("pk", "sig", "msg"))
        assert int(E.verify(pk, m, sig, E.MODE_GO_STDLIB)) == v["go"]
        assert int(E.verify(pk, m, sig, E.MODE_ZIP215)) == v["zip215"]
        ks.append(E.scalar_from_hash(E.sha512(sig[:32] + pk + m)))
    assert _windows(ks) == [v["windows"] for v in ed["raw"]]
    assert all(v["windows"] >= 35 for v in ed["raw"]) and {35, 36} <= {v["windows"] for v in ed["raw"]}
    m, off = coracle.pack_msgs(ed["msgs"])
    for mode, key in ((0, "go"), (1, "zip215")):
        got = coracle.verify_batch(ed["pk"], ed["sig"], m, off, mode)
        assert [int(x) for x in got] == [v[key] for v in ed["raw"]]


def test_sr25519_wide_verdicts_and_flags(wide):
    _, sr = wide
    ks = []
    for v in sr["raw"]:
        pk, sig, m = (bytes.fromhex(v[k]) for k in ("pk", "sig", "msg"))
        assert int(S.verify(pk, m, sig)) == v["valid"]
        ks.append(S.challenge(S.signing_context(b"", m), pk, sig[:32]))
    assert _windows(ks) == [v["windows"] for v in sr["raw"]]
    assert all(v["windows"] >= 35 for v in sr["raw"])
    m, off = coracle.pack_msgs(sr["msgs"])
    assert [int(x) for x in coracle.sr25519_verify_batch(sr["pk"], sr["sig"], m, off)] == [v["valid"] for v in sr["raw"]]


def _run(binary, arg, ed, mode):
    buf = [struct.pack("<I", len(ed["msgs"]))]
    for i, m in enumerate(ed["msgs"]):
        buf.append(bytes([mode]) + ed["pk"][i].tobytes() + ed["sig"][i].tobytes() + struct.pack("<I", len(m)) + m)
    args = [binary] + ([arg] if arg else [])
    return np.frombuffer(subprocess.run(args, input=b"".join(buf), capture_output=True, check=True,
                                        timeout=600).stdout, np.uint8)


@pytest.mark.parametrize("mode,key", [(0, "go"), (1, "zip215")])
def test_host_builds_of_device_pipelines_on_wide_vectors(wide, mode, key):
    ed, _ = wide
    want = np.array([v[key] for v in ed["raw"]], np.uint8)
    half = _run(_build(SRC, BIN, ["-std=c++17"]), "half", ed, mode)
    assert np.array_equal(half, want)
    quad = _run(_build(QSRC, QBIN, ["-std=c++20", "-pthread"]), None, ed, mode)
    assert np.array_equal(quad, want)
