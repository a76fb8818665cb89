#!/bin/bash
# round 6: polled completion of the quad kernels (tagged slices) A/B at 10k,
# three alternating rounds; latency under load without polling beside a
# pipeline (the new default) vs polling
set -o pipefail
OUT=gpurun_out/r6p
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2 3; do
  for P in 1 0; do
    CMTV_HOST_POLL=$P timeout -k 10 200 python -u tools/vc10k_ab.py 300 > "$OUT/vc10k_poll${P}_r$R.json" 2> "$OUT/vc10k_poll${P}_r$R.err" || { tail "$OUT/vc10k_poll${P}_r$R.err"; exit 1; }
    echo "poll=$P round $R $(tail -1 "$OUT/vc10k_poll${P}_r$R.json")"
  done
done
run() {  # run <name> [env...]
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/lat_load.py 1000 > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail "$OUT/$name.err"; exit 1; }
  echo "$name $(tail -1 "$OUT/$name.json")"
}
run default
run loadpoll CMTV_LOAD_POLL=1
run default_krow CMTV_LOAD_FORM=0
run default_again
