#!/bin/bash
# round 6: latency under load with the latency forms' wave priority raised
# (s_setprio 2) -- masked / masked + idle form / unmasked -- plus a trace of the
# default and the headline's quick line (the priority must not cost it)
set -o pipefail
OUT=gpurun_out/r6i
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> [env...]
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail "$OUT/$name.err"; exit 1; }
  echo "$name $(tail -1 "$OUT/$name.json")"
}
run prio_mask_kquad
run prio_mask_krow CMTV_LOAD_FORM=0
run prio_nomask CMTV_LAT_WINDOW_MS=0
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- python3 tools/lat_trace.py "$OUT/trace_windows.json" 300 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-latency --no-sr25519 --no-light --no-c3 --steps 20 > "$OUT/quick.json" 2> "$OUT/quick.err" || { tail "$OUT/quick.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/quick.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])"
