#!/bin/bash
# A/B of the single-commit staging forms on one box, alternating rounds:
# verify_commit_10k (generic) / latency_150 (tools/vc10k_ab.py) and
# verify_commit_10k_keyset (tools/lat_load.py's first line) with KNOB=A / B.
set -o pipefail
KNOB=${KNOB:-CMTV_EARLY_SIGS}
for r in 1 2 3; do
  for v in ${A:-1} ${B:-0}; do
    env "$KNOB=$v" timeout -k 10 120 python -u tools/vc10k_ab.py > gpurun_out/ab_tmp.txt 2>/dev/null || exit 1
    env "$KNOB=$v" timeout -k 10 120 python -u -c "
import json, bench
print(json.dumps(bench.verify_commit_10k_keyset(0, 300)))" > gpurun_out/ab_tmp2.txt 2>/dev/null || exit 1
    echo "$KNOB=$v $(cat gpurun_out/ab_tmp.txt) keyset10k=$(python3 -c "import json;d=json.loads(open('gpurun_out/ab_tmp2.txt').read().strip().splitlines()[-1]);print(d['p50_ms'], d['kernel_ms'])")" >> gpurun_out/early_ab.txt
  done
done
