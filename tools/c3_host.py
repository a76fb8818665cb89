"""configs[2] through cmtv_verify_commits from host memory (bench.py
c3_host_line) on its own: python tools/c3_host.py [heights] [kinds]
(CMTV_HOST_PHASES=1 prints the host phase split at context close)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from cometbft_amd import Context  # noqa: E402

heights = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
kinds = tuple(int(k) for k in sys.argv[2].split(",")) if len(sys.argv) > 2 else (0, 1)
steps = int(os.environ.get("C3_STEPS", "3"))
ctx = Context(device=0)
ctx.keyset_cache(4)
print(json.dumps(bench.c3_host_line(ctx, 0, n_heights=heights, steps=steps, kinds=kinds)), flush=True)
ctx.close()
