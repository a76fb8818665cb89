#!/bin/bash
# round 6: full GPU suite + a bench line without the slow side lines
set -o pipefail
OUT=gpurun_out/r6b
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-sr25519 --no-light --no-c3 --steps 20 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
tail -c 3000 "$OUT/bench.json"
[ $rc -eq 0 ] || exit $rc
CMTV_LIBRARY=$PWD/tools/probe/libprobe.so timeout -k 10 300 python -u tools/keyed_phase.py > "$OUT/keyed_phase.txt" 2>&1
rc=$?
cat "$OUT/keyed_phase.txt"
exit $rc
