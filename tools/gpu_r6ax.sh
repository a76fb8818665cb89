#!/bin/bash
# round 6: final tree: the whole GPU suite, then the default bench line
set -o pipefail
OUT=gpurun_out/r6ax
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
tail -c 3000 "$OUT/bench.json"
