#!/bin/bash
# round 6: chunk submission split (bulk_prepare outside the context lock) --
# GPU tests (commit, pipeline, sanitizers), latency under load x3, c3 host
set -o pipefail
OUT=gpurun_out/r6ak
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_commit_gpu.py tests/test_pipeline_gpu.py tests/test_sanitizers.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
for R in 1 2 3; do
  timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_$R.json" 2> "$OUT/lat_$R.err" || { tail "$OUT/lat_$R.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/lat_$R.json').read().strip().splitlines()[-1])['latency_150_under_load'];print('lat $R', d['idle_p99_ms'], d['idle_spaced_p99_ms'], d['p50_ms'], d['p99_ms'], d['p99_over_idle_p99'], d['p99_over_idle_spaced_p99'], d['load_verifs_per_s_during_window'])"
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-latency --no-sr25519 --no-light --no-keyset --no-c3 --steps 5 > "$OUT/b.json" 2> "$OUT/b.err" || { tail "$OUT/b.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]);h=d['replay_c3_host'];print('c3h', h['verify_commit']['ms_per_pass'], h['verify_commit']['value'], h['verify_commit_light']['ms_per_pass'], h['packed']['verify_commit']['ms_per_pass'])"
