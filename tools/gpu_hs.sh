#!/bin/bash
# helper-summed quad kernel: parity subset, phase probe, sweep of the
# helper's share of [u]B (PRES="5 6 7": CMTV_HS_PRE).
set -o pipefail
bash tools/gpu_quick.sh tests/test_gpu_parity.py tests/test_baseline_configs_gpu.py tests/test_wide_gpu.py || exit 1
CMTV_LIBRARY=$PWD/tools/probe/libprobe.so timeout -k 10 120 python tools/phase_probe.py > gpurun_out/phase_hs.log 2>&1 || { tail gpurun_out/phase_hs.log; exit 1; }
grep -v amdgpu gpurun_out/phase_hs.log | python3 -c "
import sys,json
for l in sys.stdin:
    k,v=l.split(' ',1); d=json.loads(v)
    print(k, {x:d[x] for x in ('end_median','end_max','quads_wait_at_b1_for_helper','quads_wait_at_b2_for_helper','helper_b1_median','quad_b1_median','quad_b2_median','hs_helper_window_wait_median','hs_quad_window_wait_median')})
"
for pre in ${PRES:-4 5 6}; do CMTV_HS_PRE=$pre timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-c3 --no-light --no-sr25519 --no-latency > gpurun_out/hs_$pre.json 2>/dev/null || exit 1; python3 -c "import json; d=json.loads(open('gpurun_out/hs_$pre.json').read().strip().splitlines()[-1]); print('pre $pre', d['value'], 'kms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'zip kms', d['zip215']['kernel_ms'], 'ok', d['config']['verdicts_ok'])"; done
