import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(autouse=True)
def _torch_cuda_first(request):
    """GPU tests: torch initialises HIP before libcmtverify does. torch's wheel
    carries its own HIP runtime; opened second it finds no device ("No HIP
    GPUs are available") in a process where the library's runtime came first."""
    if request.node.get_closest_marker("gpu"):
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    yield


@pytest.fixture(scope="session")
def corpus():
    with open(os.path.join(ROOT, "tests", "golden", "corpus.json")) as f:
        doc = json.load(f)
    vecs = doc["vectors"]
    pk = np.array([np.frombuffer(bytes.fromhex(v["pk"]), np.uint8) for v in vecs])
    sig = np.array([np.frombuffer(bytes.fromhex(v["sig"]), np.uint8) for v in vecs])
    msgs = [bytes.fromhex(v["msg"]) for v in vecs]
    go = np.array([v["go"] for v in vecs], np.uint8)
    zip215 = np.array([v["zip215"] for v in vecs], np.uint8)
    cats = [v["cat"] for v in vecs]
    return {"pk": pk, "sig": sig, "msgs": msgs, "go": go, "zip215": zip215, "cats": cats}


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cometbft_amd import Context

    return Context(device=0)


@pytest.fixture(scope="session")
def gpu_ctx_lane():
    """A context that always uses the one-signature-per-lane kernels
    (CMTV_QUAD_MAX=0, CMTV_KEYED_QUAD_MAX=0), so small batches exercise both
    kernel shapes."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cometbft_amd import Context

    old = {k: os.environ.get(k) for k in ("CMTV_QUAD_MAX", "CMTV_KEYED_QUAD_MAX")}
    for k in old:
        os.environ[k] = "0"
    try:
        return Context(device=0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="session")
def gpu_ctx_quad():
    """A context whose small Ed25519 batches take the 4-lanes-per-signature
    kernel (CMTV_OCT_MAX=0) instead of the default 8-lane one (oct.h)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cometbft_amd import Context

    old = os.environ.get("CMTV_OCT_MAX")
    os.environ["CMTV_OCT_MAX"] = "0"
    try:
        return Context(device=0)
    finally:
        if old is None:
            del os.environ["CMTV_OCT_MAX"]
        else:
            os.environ["CMTV_OCT_MAX"] = old


def _env_ctx(**env):
    """A Context opened with the CMTV_* knobs in env set (then restored)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cometbft_amd import Context

    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return Context(device=0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="session")
def gpu_ctx_lane256():
    """The lane kernels (as gpu_ctx_lane) with registered keys' [s]B over the
    B table's radix-256 comb (CMTV_KEYED_MIXED=0) instead of its radix-2^16
    comb (keyed_lane.hip kComb256 vs kCombMixed)."""
    return _env_ctx(CMTV_QUAD_MAX=0, CMTV_KEYED_QUAD_MAX=0, CMTV_KEYED_MIXED=0)


@pytest.fixture(scope="session")
def gpu_ctx_quad2s():
    """Small Ed25519 batches on the helper-wave quad kernel whose quads add
    both table entries of every window themselves (k_verify_quad_split,
    CMTV_QUAD_HS=0) instead of its helper-summed form (k_verify_quad_hs)."""
    return _env_ctx(CMTV_OCT_MAX=0, CMTV_QUAD_HS=0)


@pytest.fixture(scope="session")
def gpu_ctx_oct2():
    """Small Ed25519 batches on the two-wave oct kernel (CMTV_ROW_MAX=0)
    instead of the default one-signature-per-wave row kernel (row.h)."""
    return _env_ctx(CMTV_ROW_MAX=0)


@pytest.fixture(scope="session")
def gpu_ctx_row():
    """Ed25519 batches up to 4,000 signatures on the one-wave row kernel
    (k_verify_row_split: several rounds of 768), so the corpus and every
    ragged size run through it."""
    return _env_ctx(CMTV_ROW_MAX=4000, CMTV_ROW2_MAX=0)


@pytest.fixture(scope="session")
def gpu_ctx_row2():
    """The same on the two-wave row kernel (k_verify_row2_split: one
    signature per workgroup, rounds of 256)."""
    return _env_ctx(CMTV_ROW_MAX=4000, CMTV_ROW2_MAX=4000, CMTV_ROW_WAVES=2)


@pytest.fixture(scope="session")
def gpu_ctx_row4():
    """The same on the four-wave row kernel (k_verify_row4_split), the
    default at 256 signatures and below."""
    return _env_ctx(CMTV_ROW_MAX=4000, CMTV_ROW2_MAX=4000, CMTV_ROW_WAVES=4)


@pytest.fixture(scope="session")
def gpu_ctx_krow():
    """Registered-key batches up to 4,000 on the keyed row kernel
    (k_verify_keyed_row_split), so the corpus runs through it."""
    return _env_ctx(CMTV_KEYED_ROW_MAX=4000)


@pytest.fixture(scope="session")
def gpu_ctx_kquad2():
    """Small registered-key batches on the two-helper keyed quad kernel
    (CMTV_KEYED_ROW_MAX=0) instead of the default keyed row kernel."""
    return _env_ctx(CMTV_KEYED_ROW_MAX=0)


@pytest.fixture(scope="session")
def gpu_ctx_oct1():
    """A context whose small Ed25519 batches take the one-wave oct kernel
    (CMTV_OCT_SPLIT_MAX=0) instead of the default two-wave form."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cometbft_amd import Context

    old = os.environ.get("CMTV_OCT_SPLIT_MAX")
    os.environ["CMTV_OCT_SPLIT_MAX"] = "0"
    try:
        return Context(device=0)
    finally:
        if old is None:
            del os.environ["CMTV_OCT_SPLIT_MAX"]
        else:
            os.environ["CMTV_OCT_SPLIT_MAX"] = old


@pytest.fixture(scope="session")
def gpu_ctx_quad1():
    """Small Ed25519 batches on the one-wave quad kernel (CMTV_OCT_MAX=0,
    CMTV_QUAD_SPLIT_MAX=0) instead of its helper-wave form."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cometbft_amd import Context

    keys = ("CMTV_OCT_MAX", "CMTV_QUAD_SPLIT_MAX")
    old = {k: os.environ.get(k) for k in keys}
    for k in keys:
        os.environ[k] = "0"
    try:
        return Context(device=0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
