#!/bin/bash
# Full GPU pass: parity tests, smoke, PMC traffic passes, bench, rocprof kernel stats.
# Usage (via gpurun): bash tools/gpu_full.sh [tag]
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$OUT/$name.log"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
QUICK="--no-cpu-baseline --no-latency --no-sr25519"
if [ -z "$SKIP_PMC" ]; then
  step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py $QUICK --steps 5 --warmup 1 ${BENCH_ARGS}
  step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py $QUICK --steps 5 --warmup 1 ${BENCH_ARGS}
  step pmc_sq 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py $QUICK --steps 5 --warmup 1 ${BENCH_ARGS}
  python3 tools/traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" profiles/r01_traffic.json > "$OUT/traffic.log" 2>&1 || { cat "$OUT/traffic.log"; exit 1; }
fi
step bench 900 python bench.py ${BENCH_ARGS}
cp "$OUT/bench.log" "$OUT/bench.json"
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py $QUICK ${BENCH_ARGS}
echo "done $TAG"
