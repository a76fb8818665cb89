#!/bin/bash
# Sweep of a runtime knob on one box, alternating values each round:
# the configs[1] step's kernel time in both modes (bench.py quick form).
#   KNOB=CMTV_HS_PRE VALS="6 7 8" ROUNDS=2 bash tools/gpu_knob_sweep.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/knob_sweep
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VALS; do
    env "$KNOB=$v" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-light --no-sr25519 --no-latency > "$OUT/b_${v}_$r.json" 2> "$OUT/b_${v}_$r.err" || { tail -20 "$OUT/b_${v}_$r.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$KNOB=$v', d['value'], 'kms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'zip kms', d['zip215']['kernel_ms'], d['zip215']['frac'], 'ok', d['config']['verdicts_ok'])" | tee -a "$OUT/summary.txt"
  done
done
