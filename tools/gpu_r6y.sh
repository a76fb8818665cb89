#!/bin/bash
# round 6: keyed zero-copy on by default -- the whole GPU suite, then three
# more alternating A/B rounds against CMTV_KEYED_ZC=0
set -o pipefail
OUT=gpurun_out/r6y
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.txt" 2>&1 || { tail -40 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
for R in 1 2 3; do
  for Z in 1 0; do
    CMTV_KEYED_ZC=$Z timeout -k 10 200 python -u tools/vc10k_ab.py 300 > "$OUT/zc${Z}_r$R.json" 2> "$OUT/zc${Z}_r$R.err" || { tail "$OUT/zc${Z}_r$R.err"; exit 1; }
    echo "keyed_zc=$Z round $R $(tail -1 "$OUT/zc${Z}_r$R.json")"
  done
done
timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/lat.json" 2> "$OUT/lat.err" || { tail "$OUT/lat.err"; exit 1; }
tail -1 "$OUT/lat.json"
