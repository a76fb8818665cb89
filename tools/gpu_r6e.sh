#!/bin/bash
# round 6: speculative VerifyCommit (GPU parity + 10k keyset A/B), latency under
# load with 1 ms-spaced calls (masked / masked+idle form / unmasked), host ceiling x3
set -o pipefail
OUT=gpurun_out/r6e
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_commit_gpu.py -k "spec or stale or keyset" > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -3 "$OUT/tests.txt"
timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_default.json" 2> "$OUT/lat_default.err" || exit 1
cat "$OUT/lat_default.json"
CMTV_SPEC=0 CMTV_LOAD_FORM=0 timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_nospec_idleform.json" 2> "$OUT/lat_nospec_idleform.err" || exit 1
cat "$OUT/lat_nospec_idleform.json"
CMTV_LAT_WINDOW_MS=0 timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat_nomask.json" 2> "$OUT/lat_nomask.err" || exit 1
cat "$OUT/lat_nomask.json"
for R in 1 2 3; do for K in 0 1; do timeout -k 10 120 ./tests/host/pipebench 100000 16 $K 1048576 150 1 0 8 1; done; done > "$OUT/pipebench.txt" 2>&1 || exit 1
grep -i "ms/pass\|per pass\|pass" "$OUT/pipebench.txt" | head -20
