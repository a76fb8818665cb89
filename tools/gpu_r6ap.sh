#!/bin/bash
# round 6: the loaded call's device time -- staging read in place over PCIe
# (default) vs copied first (CMTV_KEYED_ZC=0 CMTV_LOAD_ZC=0), alternating
set -o pipefail
OUT=gpurun_out/r6ap
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2; do
  for Z in 1 0; do
    CMTV_KEYED_ZC=$Z CMTV_LOAD_ZC=$Z CMTV_CALL_TRACE=2 timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_${Z}_$R.json" 2> "$OUT/lat_${Z}_$R.err" || { tail "$OUT/lat_${Z}_$R.err"; exit 1; }
    python3 -c "import json;L=open('$OUT/lat_${Z}_$R.json').read().strip().splitlines();d=json.loads(L[-1])['latency_150_under_load'];print('zc $Z round $R load', d['idle_p50_ms'], d['idle_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'])"
    grep cmtv_call_trace "$OUT/lat_${Z}_$R.err" | tail -1 | cut -c1-330
  done
done
