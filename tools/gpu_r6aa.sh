#!/bin/bash
# round 6: the pipeline's host pool at 13 vs 16 threads under a 16-CPU quota
# (headroom for the latency thread) -- under load and at 10k, alternating
set -o pipefail
OUT=gpurun_out/r6aa
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2 3; do
  for W in 16 13; do
    CMTV_HOST_THREADS=$W timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_${W}_$R.json" 2> "$OUT/lat_${W}_$R.err" || { tail "$OUT/lat_${W}_$R.err"; exit 1; }
    python3 -c "import json;L=open('$OUT/lat_${W}_$R.json').read().strip().splitlines();k=json.loads(L[0])['verify_commit_10k_keyset'];d=json.loads(L[-1])['latency_150_under_load'];print('threads $W round $R keyset', k['p50_ms'], k['pinned']['p50_ms'], 'load', d['idle_p50_ms'], d['idle_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'])"
  done
done
