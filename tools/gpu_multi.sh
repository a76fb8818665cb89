#!/bin/bash
# runtime GPU tests + the N=2 bench flow rehearsed on one GPU (repeated ordinal)
set -o pipefail
OUT=gpurun_out/multi
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_runtime_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -5 "$OUT/pytest.log"
QUICK="--no-cpu-baseline --no-latency --no-sr25519 --no-light --no-c3 --steps 50 --warmup 5"
timeout -k 10 300 python bench.py $QUICK > "$OUT/bench1.json" 2> "$OUT/bench1.err" || { tail -20 "$OUT/bench1.err"; exit 1; }
cat "$OUT/bench1.json"
CMTV_BENCH_DEVICES=0,0 timeout -k 10 300 python bench.py --gpus 2 $QUICK > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { tail -20 "$OUT/bench2.err"; exit 1; }
cat "$OUT/bench2.json"
