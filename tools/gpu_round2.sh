#!/bin/bash
# full GPU pass: tests + smoke, then the default bench line
set -o pipefail
OUT=gpurun_out/r2
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -5 "$OUT/bench.err"; cat "$OUT/bench.json"; exit $rc
