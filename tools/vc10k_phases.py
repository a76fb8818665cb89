"""Host phases of one 10k keyset-cache VerifyCommit (bench verify_commit_10k_keyset,
heap and pinned), from the library's phase clock (CMTV_HOST_PHASES=1 prints
per-call microseconds at cmtv_close):
  CMTV_HOST_PHASES=1 python tools/vc10k_phases.py [iters]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["CMTV_HOST_PHASES"] = "1"

import bench  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
print(json.dumps({"verify_commit_10k_keyset": bench.verify_commit_10k_keyset(0, iters)}), flush=True)
