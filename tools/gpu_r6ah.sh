#!/bin/bash
# round 6: keyed bulk verdicts stored by the kernel into mapped host memory (CMTV_BULK_BM_DIRECT) -- pipeline
# GPU tests, then replay_c3_host A/B, alternating
set -o pipefail
OUT=gpurun_out/r6ah
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_pipeline_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
for R in 1 2; do
  for P in 1 0; do
    CMTV_BULK_BM_DIRECT=$P timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-latency --no-sr25519 --no-light --no-keyset --no-c3 --steps 5 > "$OUT/b_${P}_$R.json" 2> "$OUT/b_${P}_$R.err" || { tail "$OUT/b_${P}_$R.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/b_${P}_$R.json').read().strip().splitlines()[-1]);h=d['replay_c3_host'];print('bmdirect $P round $R', h['verify_commit']['ms_per_pass'], h['verify_commit']['value'], h['verify_commit_light']['ms_per_pass'], h['packed']['verify_commit']['ms_per_pass'])"
  done
done
