#!/bin/bash
# A/B of the helper's comb positions before barrier 1 (CMTV_HS_PRE) on the
# resident headline and the node-shaped verify_commit_10k (zero-copy staged
# sign-bytes inputs delay the helper's start). Usage (via gpurun):
#   VALUES="6 3 6 3" bash tools/hs_pre_ab.sh
set -o pipefail
OUT=gpurun_out/hs_pre_ab.txt
: > "$OUT"
for v in ${VALUES:-6 4 3 2 6}; do
  CMTV_HS_PRE=$v timeout -k 10 200 python bench.py --steps 30 --no-c3 --no-light --no-keyset --no-latency \
    --no-cpu-baseline --no-sr25519 > gpurun_out/hs_pre_$v.json 2> gpurun_out/hs_pre_$v.err || exit 1
  CMTV_HS_PRE=$v timeout -k 10 200 python tools/vc10k_ab.py > gpurun_out/hs_pre_vc_$v.json 2>> gpurun_out/hs_pre_$v.err || exit 1
  python3 - "$v" >> "$OUT" <<'PY' || exit 1
import json, sys
v = sys.argv[1]
d = [json.loads(l) for l in open(f"gpurun_out/hs_pre_{v}.json") if l.startswith("{")][-1]
vc = [json.loads(l) for l in open(f"gpurun_out/hs_pre_vc_{v}.json") if l.startswith("{")][-1]
print(json.dumps({"hs_pre": v, "headline_ms": d["ms_per_step"], "zip215_ms": d["zip215"]["ms_per_step"],
                  "e2e_10k": d["e2e_10k"]["ms"], "vc10k_p50": vc["vc10k_p50"], "vc10k_kernel": vc["vc10k_kernel"]}))
PY
  tail -1 "$OUT"
done
