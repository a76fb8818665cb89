#!/bin/bash
# Round-4 headline evidence: rocprofv3 kernel-trace stats
# of the default bench's quick form, and separate --pmc passes over the same
# command -- FETCH_SIZE, WRITE_SIZE, and two SQ groups -- so bench.py's
# roofline.traffic and valu_utilisation come from this round's kernels.
# Usage (via gpurun): TAG=r04 [KERNEL=k_verify_quad_hs] bash tools/gpu_prof_r04.sh
# (the traffic of KERNEL<0u> / <1u> merged into $OUT/traffic.json, bench.py's
# PMC_TRAFFIC format)
set -o pipefail
TAG=${TAG:-r04}
KERNEL=${KERNEL:-k_verify_quad_hs}
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
step stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 bench.py $QUICK
step pmc_fetch 120 timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py $QUICK
step pmc_write 120 timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py $QUICK
step pmc_sq1 120 timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d "$OUT/pmc_sq1" -o run -- python3 bench.py $QUICK
step pmc_sq2 120 timeout -s KILL 110 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_sq2" -o run -- python3 bench.py $QUICK
python3 tools/pmc_summary.py "$OUT/pmc_sq.txt" $(dirname $(find "$OUT/pmc_sq1" -name '*counter_collection.csv' | head -1)) $(dirname $(find "$OUT/pmc_sq2" -name '*counter_collection.csv' | head -1)) > /dev/null 2>&1 || echo "pmc summary failed"
for k in '<0u>' '<1u>'; do
  python3 tools/traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/traffic_${k:1:1}.json" "$KERNEL$k" > "$OUT/traffic_${k:1:1}.log" 2>&1 || { cat "$OUT/traffic_${k:1:1}.log"; exit 1; }
  cat "$OUT/traffic_${k:1:1}.log"
done
python3 - "$OUT" "$KERNEL" "$QUICK" <<'PY'
import json, sys
out, kern, quick = sys.argv[1:4]
go = json.load(open(f"{out}/traffic_0.json")); zp = json.load(open(f"{out}/traffic_1.json"))
doc = {"go": go, "zip215": zp,
       "command": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) -- python3 bench.py {quick} (tools/gpu_prof_r04.sh)",
       "bytes_per_launch": go["bytes_per_launch"], "kernel": go["kernel"]}
json.dump(doc, open(f"{out}/traffic.json", "w"), indent=1)
PY
echo done
