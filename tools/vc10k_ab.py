"""verify_commit_10k (generic kernels) and latency_150 (C call) p50s on this
box, for A/Bs of host-path knobs: CMTV_EARLY_SIGS=0 python tools/vc10k_ab.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cometbft_amd import Context  # noqa: E402

ctx = Context(device=0)
r = bench.verify_commit_10k(ctx, 0, 300)
l150 = bench.latency_150(ctx, 0, 1000)
print(json.dumps({"early": os.environ.get("CMTV_EARLY_SIGS", "1"), "vc10k_p50": r["p50_ms"], "vc10k_p99": r["p99_ms"],
                  "vc10k_kernel": r["kernel_ms"], "l150_p50": l150["p50_ms"], "l150_p99": l150["p99_ms"],
                  "l150_keyset_p50": l150["keyset_cache"]["p50_ms"]}), flush=True)
