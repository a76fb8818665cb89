"""bench.py's latency_150_under_load and verify_commit_10k_keyset lines on
their own: python tools/lat_load.py [iters]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
print(json.dumps({"verify_commit_10k_keyset": bench.verify_commit_10k_keyset(0, 200)}), flush=True)
print(json.dumps({"latency_150_under_load": bench.latency_150_under_load(0, iters)}), flush=True)
