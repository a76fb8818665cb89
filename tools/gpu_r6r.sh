#!/bin/bash
# round 6: rocprof evidence of this round's headline (TAG=r06: kernel stats,
# FETCH/WRITE and SQ passes) and the host ceiling (pipebench, with the cut phase)
set -o pipefail
mkdir -p gpurun_out/r6r
export TMPDIR=/tmp
for R in 1 2; do for K in 0 1; do timeout -k 10 120 ./tests/host/pipebench 100000 16 $K 1048576 150 1 0 8 1; done; done > gpurun_out/r6r/pipebench.txt 2>&1 || { cat gpurun_out/r6r/pipebench.txt; exit 1; }
cat gpurun_out/r6r/pipebench.txt
TAG=r06 bash tools/gpu_prof_r04.sh
