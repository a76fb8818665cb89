#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/dbg/quad_debug > gpurun_out/qd_time.txt 2>&1 || { cat gpurun_out/qd_time.txt; exit 1; }
grep cycles gpurun_out/qd_time.txt
bash tools/gpu_bench.sh || exit 1
timeout -k 10 400 python tools/crossover.py > gpurun_out/crossover.json 2> gpurun_out/crossover.err || { tail gpurun_out/crossover.err; exit 1; }
cat gpurun_out/crossover.json
