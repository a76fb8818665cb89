#!/bin/bash
# round 6: CMTV_PREP_STREAM 1 vs 0 (a fifth hardware queue per lane) under load,
# three alternating rounds
set -o pipefail
OUT=gpurun_out/r6ar
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2 3; do
  for P in 1 0; do
    CMTV_PREP_STREAM=$P timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_${P}_$R.json" 2> "$OUT/lat_${P}_$R.err" || { tail "$OUT/lat_${P}_$R.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/lat_${P}_$R.json').read().strip().splitlines()[-1])['latency_150_under_load'];print('prep $P round $R', d['idle_p99_ms'], d['idle_spaced_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'], d['load_verifs_per_s_during_window'])"
  done
done
