#!/bin/bash
# round 6: device-event split of the loaded call (CMTV_CALL_TRACE) --
# keyed / commit GPU tests, then the traced latency-under-load line x2
set -o pipefail
OUT=gpurun_out/r6ao
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2; do
  CMTV_CALL_TRACE=2 timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_$R.json" 2> "$OUT/lat_$R.err" || { tail "$OUT/lat_$R.err"; exit 1; }
  python3 -c "import json;L=open('$OUT/lat_$R.json').read().strip().splitlines();k=json.loads(L[0])['verify_commit_10k_keyset'];d=json.loads(L[-1])['latency_150_under_load'];print('lat $R keyset', k['p50_ms'], k['kernel_ms'], k['pinned']['p50_ms'], 'load', d['idle_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'])"
  grep cmtv_call_trace "$OUT/lat_$R.err" | tail -1 | cut -c1-400
done
