#!/bin/bash
# round 6: lock handoff (bulk_relock) -- pipeline/commit GPU tests, latency
# under load twice, replay_c3_host not regressed
set -o pipefail
OUT=gpurun_out/r6t
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_commit_gpu.py tests/test_pipeline_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for R in 1 2; do
  timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_$R.json" 2> "$OUT/lat_$R.err" || { tail "$OUT/lat_$R.err"; exit 1; }
  echo "lat $R $(tail -1 "$OUT/lat_$R.json")"
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-latency --no-sr25519 --no-light --no-keyset --no-c3 --steps 20 > "$OUT/quick.json" 2> "$OUT/quick.err" || { tail "$OUT/quick.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/quick.json').read().strip().splitlines()[-1]);h=d.get('replay_c3_host',{});print(d['value'],d['ms_per_step'],d['roofline']['frac'],h.get('verify_commit',{}).get('value'),h.get('verify_commit_light',{}).get('value'))"
