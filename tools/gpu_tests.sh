#!/bin/bash
# GPU test pass: pytest -m gpu (optionally a subset: bash tools/gpu_tests.sh tests/test_x.py ...) + smoke.
set -o pipefail
OUT=gpurun_out/tests
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${@:-tests}
timeout -k 10 900 python -u -m pytest $ARGS -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -30 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "!! pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
