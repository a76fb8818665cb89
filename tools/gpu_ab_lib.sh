#!/bin/bash
# A/B of two builds on one box: tools/probe/libold.so vs the in-tree library,
# alternating, the configs[1] step's kernel time in both modes (bench.py
# quick form); then the quad phase probe of tools/probe/libprobe.so.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab_lib
mkdir -p "$OUT"
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export CMTV_LIBRARY=$PWD/tools/probe/libold.so; else unset CMTV_LIBRARY; fi
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-light --no-sr25519 --no-latency > "$OUT/b_${v}_$r.json" 2> "$OUT/b_${v}_$r.err" || { tail -20 "$OUT/b_${v}_$r.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], 'kms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'zip kms', d['zip215']['kernel_ms'], 'ok', d['config']['verdicts_ok'])"
  done
done
unset CMTV_LIBRARY
if [ -z "$NO_PROBE" ]; then
  CMTV_LIBRARY=$PWD/tools/probe/libprobe.so timeout -k 10 120 python tools/phase_probe.py > "$OUT/phase.log" 2>&1 || { tail "$OUT/phase.log"; exit 1; }
  grep -v amdgpu "$OUT/phase.log" | python3 -c "
import sys,json
for l in sys.stdin:
    k,v=l.split(' ',1); d=json.loads(v)
    print(k, {x:d[x] for x in ('end_median','end_max','helper_b1_median','quad_b1_median','quad_b2_median','hs_helper_window_wait_median','hs_quad_window_wait_median')})
"
fi
