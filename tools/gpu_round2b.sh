#!/bin/bash
# GPU tests, then the profile set (tools/gpu_prof.sh), then an sr25519 timing
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2b
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -B5 -A40 "FAIL\|Error" "$OUT/pytest.log" | head -100; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency --no-c3 --no-light > "$OUT/bench_sr.json" 2> "$OUT/bench_sr.err" || { tail -20 "$OUT/bench_sr.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench_sr.json').read().strip().splitlines()[-1]); print('headline', d['value'], d['roofline']['frac'], 'sr', d['sr25519']['value'], d['sr25519']['kernel_ms'])"
TAG=${TAG:-r02d} bash tools/gpu_prof.sh
