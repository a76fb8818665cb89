#!/bin/bash
# GPU tests, then a short bench (latency lines incl. the keyset cache)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${ITER:-iter4}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -B5 -A40 "FAIL\|Error" "$OUT/pytest.log" | head -100; exit $rc; }
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-light > "$OUT/b.json" 2> "$OUT/b.err" || { tail -20 "$OUT/b.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('headline', d['value'], d['roofline']['frac']); print('lat', d['latency_150']['p50_ms'], 'keyset', d['latency_150']['keyset_cache']); print('replay', d['replay_150'])"
