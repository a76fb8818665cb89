#!/bin/bash
# round 6: is the residual under-load tail CPU-quota pressure from the
# pipeline's 16 host workers? host threads 16 vs 8, alternating
set -o pipefail
OUT=gpurun_out/r6v
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2; do
  for T in 16 8; do
    CMTV_HOST_THREADS=$T timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_${T}_$R.json" 2> "$OUT/lat_${T}_$R.err" || { tail "$OUT/lat_${T}_$R.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/lat_${T}_$R.json').read().strip().splitlines()[-1])['latency_150_under_load'];print('threads $T round $R', d['idle_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'], d['load_verifs_per_s_during_window'])"
  done
done
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
