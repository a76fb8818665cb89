"""bench.py's verify_commit_10k (generic quad kernel) and
verify_commit_10k_keyset (registered-key quad kernel) lines under the current
environment -- one side of an A/B (tools/gpu_r6p.sh alternates knobs across
processes): python tools/vc10k_ab.py [iters]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
k = bench.verify_commit_10k_keyset(0, iters)
from cometbft_amd import Context  # noqa: E402

ctx = Context(device=0)
g = bench.verify_commit_10k(ctx, 0, iters)
ctx.close()
print(json.dumps({"keyset_p50": k["p50_ms"], "keyset_pinned_p50": k["pinned"]["p50_ms"],
                  "generic_p50": g["p50_ms"], "generic_pinned_p50": g.get("pinned", {}).get("p50_ms")}), flush=True)
