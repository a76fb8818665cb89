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


# The verification forms (cometbft_amd/csrc/kernels.h kForm*, kKeyed*) a
# context is forced to at every size with the CMTV_FORM debug knob, so the
# corpus and every ragged size run through each kernel the default bands
# reach (runtime.cpp ed_form / sr_form / keyed_form):
#   row4  k_verify_row4_split       (Ed25519 default <= 256)
#   row   k_verify_row_split        (<= 1,536)
#   oct2  k_verify_oct_split        (<= 2,048)
#   quad  k_verify_quad_hs          (<= 49,152; sr25519 too)
#   lane  k_verify, k_verify_sr25519 and the keyed lane kernels (above)
#   krow  k_verify_keyed_row_split  (registered keys <= 512)
#   kquad k_verify_keyed_quad_split (<= 36,864)
FORMS = {"row4": "row4", "row": "row", "oct2": "oct2", "quad": "quad", "lane": "lane,klane", "krow": "krow",
         "kquad": "kquad"}
ED_FORMS = ["row4", "row", "oct2", "quad", "lane"]


@pytest.fixture(scope="session")
def form_ctx():
    """form name -> a session Context forced to that form (CMTV_FORM)."""
    made = {}

    def get(name):
        if name not in made:
            made[name] = _env_ctx(CMTV_FORM=FORMS[name])
        return made[name]

    return get


@pytest.fixture(scope="session")
def gpu_ctx_lane(form_ctx):
    """A context that always uses the one-signature-per-lane kernels
    (CMTV_FORM=lane,klane), so small batches exercise both kernel shapes."""
    return form_ctx("lane")
