#!/bin/bash
# profiles for the round: kernel-trace stats of the default bench, PMC passes
# (FETCH/WRITE traffic, SQ instruction/cycle counters) of the headline step,
# and the quad kernel's phase cycles (s_memtime probes).
set -o pipefail
TAG=${TAG:-r02}
OUT=gpurun_out/prof_$TAG
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
QUICK="--no-cpu-baseline --no-latency --no-sr25519 --no-light --no-c3 --steps 20 --warmup 3"
step phases 120 ./tools/dbg/quad_debug
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py $QUICK
step pmc_fetch 90 timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py $QUICK
step pmc_write 90 timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py $QUICK
# SQ counters of every verify kernel (oct, quad, lane, keyed quad, keyed lane)
step kstats 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kstats" -o run -- python3 tools/pmc_driver.py
step pmc_sq1 150 timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d "$OUT/pmc_sq1" -o run -- python3 tools/pmc_driver.py
step pmc_sq2 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_sq2" -o run -- python3 tools/pmc_driver.py
python3 tools/pmc_summary.py "$OUT/pmc_sq.txt" "$OUT/pmc_sq1" "$OUT/pmc_sq2" > /dev/null 2>&1 || echo "pmc summary failed"
python3 tools/traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/traffic.json" > "$OUT/traffic.log" 2>&1 || { cat "$OUT/traffic.log"; exit 1; }
cat "$OUT/traffic.log"
echo done
