#!/bin/bash
# round 6: prep kernels on exec_masked (no fifth queue) -- pipeline tests,
# latency under load x2, replay_c3_host
set -o pipefail
OUT=gpurun_out/r6as
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_pipeline_gpu.py tests/test_commit_gpu.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
for R in 1 2; do
  timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_$R.json" 2> "$OUT/lat_$R.err" || { tail "$OUT/lat_$R.err"; exit 1; }
  python3 -c "import json;L=open('$OUT/lat_$R.json').read().strip().splitlines();k=json.loads(L[0])['verify_commit_10k_keyset'];d=json.loads(L[-1])['latency_150_under_load'];print('lat $R keyset', k['p50_ms'], k['pinned']['p50_ms'], 'load', d['idle_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'])"
done
for P in 1 0; do
  CMTV_PREP_STREAM=$P timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-latency --no-sr25519 --no-light --no-keyset --no-c3 --steps 5 > "$OUT/b_$P.json" 2> "$OUT/b_$P.err" || { tail "$OUT/b_$P.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/b_$P.json').read().strip().splitlines()[-1]);h=d['replay_c3_host'];print('c3h prep $P', h['verify_commit']['ms_per_pass'], h['verify_commit']['value'], h['verify_commit_light']['ms_per_pass'], h['packed']['verify_commit']['ms_per_pass'])"
done
