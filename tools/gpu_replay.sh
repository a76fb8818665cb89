#!/bin/bash
# replay / light-client lines with their C-call timings, plus replay GPU tests
set -o pipefail
OUT=gpurun_out/replay
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_replay_gpu.py tests/test_commit_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 400 python bench.py --no-cpu-baseline --no-sr25519 --no-c3 --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(json.dumps(d['replay_150'])); print(json.dumps(d['light_client']))"
