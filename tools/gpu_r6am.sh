#!/bin/bash
# round 6: where the loaded 150-validator call's tail goes, from the
# library's own clock (CMTV_CALL_TRACE=2: calls beside a pipeline call only)
set -o pipefail
OUT=gpurun_out/r6am
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2; do
  CMTV_CALL_TRACE=2 timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_$R.json" 2> "$OUT/lat_$R.err" || { tail "$OUT/lat_$R.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/lat_$R.json').read().strip().splitlines()[-1])['latency_150_under_load'];print('lat $R', d['idle_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'])"
  grep cmtv_call_trace "$OUT/lat_$R.err" | tail -1
done
