#!/bin/bash
# round 6: reserve 8 vs 16 CUs with the lock handoff, alternating
set -o pipefail
OUT=gpurun_out/r6u
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2; do
  for C in 16 8; do
    CMTV_LAT_RESERVE_CUS=$C timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_${C}_$R.json" 2> "$OUT/lat_${C}_$R.err" || { tail "$OUT/lat_${C}_$R.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/lat_${C}_$R.json').read().strip().splitlines()[-1])['latency_150_under_load'];print('reserve $C round $R', d['idle_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'], d['load_verifs_per_s_during_window'])"
  done
done
