#!/bin/bash
# e2e host-buffer path A/B (progressive H2D) + the large-batch GPU tests
set -o pipefail
OUT=gpurun_out/e2e
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_batch_gpu.py tests/test_baseline_configs_gpu.py tests/test_keyed_gpu.py tests/test_runtime_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-sr25519 --no-light --no-c3 --steps 20 --warmup 3 > "$OUT/b$i.json" 2> "$OUT/b$i.err" || { tail -20 "$OUT/b$i.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/b$i.json')); print(d['value'], json.dumps(d['e2e_10k']))"
done
