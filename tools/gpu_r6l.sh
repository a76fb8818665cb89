#!/bin/bash
# round 6: per-call timeline of the 10k keyset VerifyCommit (HIP API +
# copies + kernels), speculation on and off
set -o pipefail
OUT=gpurun_out/r6l
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in spec nospec; do
  if [ $V = nospec ]; then export CMTV_SPEC=0; fi
  timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace_$V" -o run -- python3 tools/vc10k_phases.py 200 > "$OUT/trace_$V.log" 2>&1 || { tail -20 "$OUT/trace_$V.log"; exit 1; }
  grep verify_commit "$OUT/trace_$V.log" | tail -1
  python3 tools/call_timeline.py "$OUT/trace_$V" keyed_quad_split 150 > "$OUT/timeline_$V.txt" 2>&1 || { cat "$OUT/timeline_$V.txt"; exit 1; }
  cat "$OUT/timeline_$V.txt"
done
