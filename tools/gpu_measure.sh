#!/bin/bash
# Round-3 measurements: the CPU/GPU crossover
# sweep, and the configs[2] kernels' memory counters -- FETCH_SIZE,
# WRITE_SIZE, L2 hits / misses -- plus their SQ counters and kernel stats, at
# configs[2]'s launch shape (262,144 signatures, 150 keys cycling).
# Usage (via gpurun): bash tools/gpu_measure.sh [tag]
set -o pipefail
TAG=${1:-r03m}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$OUT/$name.log"; exit $rc; fi
}
if [ -z "$SKIP_CROSS" ]; then
  timeout -k 10 600 python3 tools/crossover.py > "$OUT/crossover.json" 2> "$OUT/crossover.log" || { echo "!! crossover"; tail -20 "$OUT/crossover.log"; exit 1; }
  tail -2 "$OUT/crossover.log"
fi
export PMC_ONLY=${PMC_ONLY:-lane262k,keyed_lane262k}
step kstats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats" -o run -- python3 tools/pmc_driver.py
step pmc_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 tools/pmc_driver.py
step pmc_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 tools/pmc_driver.py
step pmc_tcc 150 timeout -s KILL 140 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/pmc_tcc" -o run -- python3 tools/pmc_driver.py
step pmc_sq 150 timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmc_sq" -o run -- python3 tools/pmc_driver.py
python3 tools/l2_traffic.py "$OUT/traffic.json" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_tcc" > "$OUT/traffic.log" 2>&1 || { cat "$OUT/traffic.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc_sq.txt" "$OUT/pmc_sq" > /dev/null 2>&1 || echo "pmc summary failed"
cat "$OUT/traffic.log"
echo "done $TAG"
