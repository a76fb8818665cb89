#!/bin/bash
# Quick GPU check after a kernel change: a pytest subset (default: the row,
# ring, commit and parity tests), then the 150-validator host phases.
# Usage (via gpurun): bash tools/gpu_quick.sh [pytest args...]
set -o pipefail
OUT=gpurun_out/quick
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${@:-tests/test_row_gpu.py tests/test_row_ring_gpu.py tests/test_commit_gpu.py tests/test_gpu_parity.py tests/test_keyed_gpu.py}
timeout -k 10 600 python -u -m pytest $ARGS -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -30; exit $rc; }
timeout -k 10 120 python tools/commit_phases.py --n 150 --iters 1000 > "$OUT/phases.log" 2>&1 || { tail -20 "$OUT/phases.log"; exit 1; }
grep -v amdgpu.ids "$OUT/phases.log"
