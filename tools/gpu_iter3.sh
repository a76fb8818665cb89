#!/bin/bash
# GPU tests, then the kernel-time sweep with the oct kernel on and off, then the latency probe
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/iter3
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -B5 -A40 "FAIL\|Error" "$OUT/pytest.log" | head -100; exit $rc; }
timeout -k 10 300 python tools/quad_sweep.py 150 1000 2048 3072 8192 10000 > "$OUT/sweep_oct.log" 2>&1 || { cat "$OUT/sweep_oct.log"; exit 1; }
grep -v amdgpu.ids "$OUT/sweep_oct.log"
CMTV_OCT_MAX=0 timeout -k 10 300 python tools/quad_sweep.py 150 2048 3072 12288 16384 > "$OUT/sweep_quad.log" 2>&1 || { cat "$OUT/sweep_quad.log"; exit 1; }
grep -v amdgpu.ids "$OUT/sweep_quad.log" | sed "s/^/quad2: /"
CMTV_OCT_MAX=0 CMTV_QUAD_SPLIT_MAX=0 timeout -k 10 300 python tools/quad_sweep.py 150 10000 12288 > "$OUT/sweep_quad1.log" 2>&1 || { cat "$OUT/sweep_quad1.log"; exit 1; }
grep -v amdgpu.ids "$OUT/sweep_quad1.log" | sed "s/^/quad1: /"
timeout -k 10 200 python3 tools/lat_probe.py 300 2>&1 | grep verify_commit
timeout -k 10 120 ./tools/dbg/quad_debug > "$OUT/phases.log" 2>&1; grep "^cycles" "$OUT/phases.log"
