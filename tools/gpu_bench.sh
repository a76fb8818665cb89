#!/bin/bash
# smoke + bench + rocprof kernel trace of the bench command
set -o pipefail
mkdir -p gpurun_out/prof
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { cat gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-latency > gpurun_out/bench_prof.json 2> gpurun_out/prof.err || { tail -20 gpurun_out/prof.err; exit 1; }
cat gpurun_out/bench_prof.json
find gpurun_out/prof -name "*stats*" | head
