#!/bin/bash
# Small-batch kernels (row.h: k_verify_row4/row2/row_split, k_verify_keyed_row_split):
# their GPU tests, wall / kernel timings at commit sizes, and -- with PROBE=1 and
# abtest/libprobe.so built (tools/row_phase.py) -- the phase probes.
#   gpurun -- 'bash tools/gpu_small.sh'
set -o pipefail
OUT=gpurun_out/small
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_row_gpu.py tests/test_gpu_parity.py tests/test_wide_gpu.py \
  tests/test_keyed_gpu.py tests/test_commit_gpu.py -k "row or keyed or commit" -x -q -m gpu \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/quick_time.py 150 256 768 > "$OUT/generic.txt" 2>&1 && cat "$OUT/generic.txt" || exit 1
timeout -k 10 120 python tools/keyed_small.py 150 256 > "$OUT/keyed.txt" 2>&1 && cat "$OUT/keyed.txt" || exit 1
if [ -n "$PROBE" ]; then
  CMTV_LIBRARY=$PWD/abtest/libprobe.so timeout -k 10 180 python tools/row_phase.py 150 row4 > "$OUT/phase_row4.txt" 2>&1 || exit 1
  CMTV_LIBRARY=$PWD/abtest/libprobe.so timeout -k 10 180 python tools/row_phase.py 150 krow > "$OUT/phase_krow.txt" 2>&1 || exit 1
  cat "$OUT/phase_row4.txt" "$OUT/phase_krow.txt"
fi
