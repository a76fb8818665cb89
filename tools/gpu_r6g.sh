#!/bin/bash
# round 6: latency under load with the CU mask's reserved bits one per XCD
# (stride 1) vs round 6's first layout (stride 32); trace of the default; and a
# copy/kernel trace of the 10k keyset VerifyCommit (where its 0.11 ms goes)
set -o pipefail
OUT=gpurun_out/r6g
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> [env...]
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail "$OUT/$name.err"; exit 1; }
  echo "$name $(tail -1 "$OUT/$name.json")"
}
run s1_kquad
run s1_krow CMTV_LOAD_FORM=0
run s1_krow_r16 CMTV_LOAD_FORM=0 CMTV_LAT_RESERVE_CUS=16
run s32_kquad CMTV_LAT_MASK_STRIDE=32
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- python3 tools/lat_trace.py "$OUT/trace_windows.json" 300 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
tail -1 "$OUT/trace.log"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace10k" -o run -- python3 tools/vc10k_phases.py 200 > "$OUT/trace10k.log" 2>&1 || { tail -20 "$OUT/trace10k.log"; exit 1; }
grep -v amdgpu.ids "$OUT/trace10k.log" | tail -3
