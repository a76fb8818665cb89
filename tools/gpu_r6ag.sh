#!/bin/bash
# round 6: staging slots 4 vs 3 (CMTV_PIPE_SLOTS) -- pipeline
# GPU tests, then replay_c3_host A/B, alternating
set -o pipefail
OUT=gpurun_out/r6ag
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2; do
  for P in 4 3; do
    CMTV_PIPE_SLOTS=$P timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-latency --no-sr25519 --no-light --no-keyset --no-c3 --steps 5 > "$OUT/b_${P}_$R.json" 2> "$OUT/b_${P}_$R.err" || { tail "$OUT/b_${P}_$R.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/b_${P}_$R.json').read().strip().splitlines()[-1]);h=d['replay_c3_host'];print('slots $P round $R', h['verify_commit']['ms_per_pass'], h['verify_commit']['value'], h['verify_commit_light']['ms_per_pass'], h['packed']['verify_commit']['ms_per_pass'])"
  done
done
