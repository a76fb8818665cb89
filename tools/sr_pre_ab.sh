#!/bin/bash
# A/B of the sr25519 helper's comb positions before barrier 1 (CMTV_HS_PRE;
# kHsCombPreSr = 0): the bench's sr25519 line at 0 / 1 / 2, alternating.
# Usage (via gpurun): bash tools/sr_pre_ab.sh -> gpurun_out/srpre.txt
set -o pipefail
rm -f gpurun_out/srpre.txt
for v in 0 1 2 0 1 2; do
  CMTV_HS_PRE=$v timeout -k 10 200 python bench.py --steps 20 --no-c3 --no-light --no-keyset --no-latency \
    --no-cpu-baseline > gpurun_out/srpre_$v.json 2>/dev/null || exit 1
  python3 -c "
import json
d = [json.loads(l) for l in open('gpurun_out/srpre_$v.json') if l.startswith('{')][-1]
print('hs_pre $v sr25519_ms', d['sr25519']['ms_per_step'], 'ed25519_ms', d['ms_per_step'])" >> gpurun_out/srpre.txt || exit 1
done
