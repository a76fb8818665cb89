#!/bin/bash
# A/B of a runtime knob on one box, alternating: KNOB=VAL_A vs KNOB=VAL_B,
# the configs[1] step's kernel time in both modes (bench.py quick form).
#   KNOB=CMTV_HS_PRE A=4 B=6 bash tools/gpu_knob_ab.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/knob_ab
mkdir -p "$OUT"
for r in 1 2; do
  for v in "$A" "$B"; do
    env "$KNOB=$v" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-light ${AB_ARGS:---no-sr25519 --no-latency} > "$OUT/b_${v}_$r.json" 2> "$OUT/b_${v}_$r.err" || { tail -20 "$OUT/b_${v}_$r.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$KNOB=$v', d['value'], 'kms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'zip kms', d['zip215']['kernel_ms'], d['zip215']['frac'], 'ok', d['config']['verdicts_ok'])"
  done
done
