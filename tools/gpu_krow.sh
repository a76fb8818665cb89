#!/bin/bash
# Keyed row kernel: keyed / keyset GPU tests, then the latency lines.
set -o pipefail
OUT=gpurun_out/krow
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_keyed_gpu.py tests/test_wide_gpu.py tests/test_commit_gpu.py tests/test_runtime_gpu.py tests/test_replay_gpu.py -k "keyed or keyset or row or commit or replay" -x -q \
  -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --no-c3 --no-sr25519 --no-light > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(json.dumps(d['latency_150'])); print(json.dumps(d['keyset_10k']))"
