#!/bin/bash
# A/B of the 150-validator VerifyCommit latency: tools/probe/libold.so vs the
# in-tree library, alternating (tools/commit_phases.py --n 150), then the row4
# phase probe of the probe build (tools/probe/libprobe.so).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/lat_ab
mkdir -p "$OUT"
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export CMTV_LIBRARY=$PWD/tools/probe/libold.so; else unset CMTV_LIBRARY; fi
    timeout -k 10 120 python tools/commit_phases.py --n ${LAT_N:-150} --iters 1000 > "$OUT/$v$r.log" 2>&1 || { tail -20 "$OUT/$v$r.log"; exit 1; }
    echo "$v $(grep commit_p50 "$OUT/$v$r.log" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["commit_p50_ms"], d["kernel_ms"])')"
  done
done
unset CMTV_LIBRARY
if [ -z "$NO_PROBE" ]; then
  CMTV_LIBRARY=$PWD/tools/probe/libprobe.so timeout -k 10 120 python tools/row_phase.py 150 row4 > "$OUT/phase.log" 2>&1 || { tail "$OUT/phase.log"; exit 1; }
  grep -v amdgpu "$OUT/phase.log" | cut -c1-400
fi
