#!/bin/bash
# round 6: CMTV_ONE_EXEC 1 vs 0 (three queues per lane instead of four) under load,
# three alternating rounds
set -o pipefail
OUT=gpurun_out/r6av
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2; do
  for P in 1 0; do
    CMTV_ONE_EXEC=$P timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_${P}_$R.json" 2> "$OUT/lat_${P}_$R.err" || { tail "$OUT/lat_${P}_$R.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/lat_${P}_$R.json').read().strip().splitlines()[-1])['latency_150_under_load'];print('one_exec $P round $R', d['idle_p99_ms'], d['idle_spaced_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'], d['load_verifs_per_s_during_window'])"
  done
done
