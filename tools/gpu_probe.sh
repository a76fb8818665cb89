#!/bin/bash
# Round-2 probe: VALU issue vs waves/SIMD, quad-kernel time vs n, SQ counters at 10k.
set -o pipefail
OUT=gpurun_out/probe
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -12 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; tail -40 "$OUT/$name.log"; exit $rc; fi
}
step occupancy 120 ./tools/microbench/occupancy
step sweep 300 env CMTV_QUAD_MAX=1000000000 python tools/quad_sweep.py 150 1000 2500 5000 7500 10000 12500 15000 20000 30000 40000
export CMTV_QUAD_MAX=1000000000
step pmc_sq1 90 timeout -s KILL 80 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d "$OUT/pmc_sq1" -o run -- python3 tools/quad_sweep.py 10000
step pmc_sq2 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_sq2" -o run -- python3 tools/quad_sweep.py 10000
echo done
