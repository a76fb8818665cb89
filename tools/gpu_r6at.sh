#!/bin/bash
# round 6: final tree: the whole GPU suite, then the default bench line
set -o pipefail
OUT=gpurun_out/r6at
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.txt" 2>&1 || { tail -40 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
tail -c 3000 "$OUT/bench.json"
