#!/bin/bash
# A/B of two builds on one box: abtest/libold.so vs the in-tree library,
# alternating, kernel time of the configs[1] step (go and zip215).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ITER:-ab}
mkdir -p "$OUT"
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export CMTV_LIBRARY=$PWD/abtest/libold.so; else unset CMTV_LIBRARY; fi
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-light ${AB_ARGS:---no-sr25519 --no-latency} > "$OUT/b_${v}_$r.json" 2> "$OUT/b_${v}_$r.err" || { tail -20 "$OUT/b_${v}_$r.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['value'], 'kms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'zip kms', d['zip215']['kernel_ms'], d['zip215']['frac'], 'sr kms', d.get('sr25519', {}).get('kernel_ms'), 'lat150', d.get('latency_150', {}).get('p50_ms'))"
  done
done
