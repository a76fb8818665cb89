#!/bin/bash
# iteration: quad-path GPU tests, then quad-kernel timing sweep
set -o pipefail
OUT=gpurun_out/iter
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_wide_gpu.py tests/test_keyed_gpu.py tests/test_sr25519_gpu.py tests/test_commit_gpu.py tests/test_baseline_configs_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -5 "$OUT/pytest.log"; [ $rc -eq 0 ] || { tail -60 "$OUT/pytest.log"; exit $rc; }
CMTV_QUAD_MAX=1000000000 timeout -k 10 300 python tools/quad_sweep.py ${SIZES:-150 1000 5000 10000 12500 20000} > "$OUT/sweep.log" 2>&1 || { cat "$OUT/sweep.log"; exit 1; }
grep -v amdgpu.ids "$OUT/sweep.log"
