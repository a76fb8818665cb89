#!/bin/bash
# A/B of the pipeline's ramp (pipeline.cpp ramp_sh) on one box, alternating:
# tools/c3_host.py (100k x 150, VerifyCommit) per variant. Round 5 used a
# temporary CMTV_PIPE_RAMP list of shifts ("3,2,1", "4,2,1", ...; empty = no
# ramp) patched into pipeline.cpp; the result is the constant there.
set -o pipefail
for r in 1 2; do
for v in "3,2,1" "4,1" "3,1" "4,2,1" "x"; do
  if [ "$v" = "x" ]; then export CMTV_PIPE_RAMP=""; else export CMTV_PIPE_RAMP="$v"; fi
  C3_STEPS=5 timeout -k 10 120 python -u tools/c3_host.py 100000 0 > gpurun_out/ramp_$r.txt.tmp 2>&1 || exit 1
  echo "ramp=$v $(grep -o '"ms_per_pass": [0-9.]*, "ms_min": [0-9.]*' gpurun_out/ramp_$r.txt.tmp)" >> gpurun_out/ramp_ab.txt
done
done
