#!/bin/bash
# New-test pass (no -x), then the whole GPU suite if nothing crashed.
# Usage: bash tools/gpu_new.sh tests/test_a.py tests/test_b.py
OUT=gpurun_out/new
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "$@" -v -m gpu --timeout 120 --timeout-method thread > "$OUT/new.log" 2>&1
rc=$?
tail -40 "$OUT/new.log"
# 0 = passed, 1 = test failures: anything else (crash, timeout) stops here
[ $rc -le 1 ] || { echo "!! new tests rc=$rc"; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > "$OUT/full.log" 2>&1
rc2=$?
tail -15 "$OUT/full.log"
echo "new rc=$rc full rc=$rc2"
exit $(( rc > rc2 ? rc : rc2 ))
