#!/bin/bash
# fused sign-bytes: commit GPU tests + configs tests + latency A/B
set -o pipefail
OUT=gpurun_out/fuse
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_commit_gpu.py tests/test_baseline_configs_gpu.py tests/test_replay_gpu.py tests/test_runtime_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -60 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
Q="--no-cpu-baseline --no-sr25519 --no-light --no-c3 --steps 50 --warmup 5"
timeout -k 10 300 python bench.py $Q > "$OUT/bench_fused.json" 2> "$OUT/bench_fused.err" || { tail -20 "$OUT/bench_fused.err"; exit 1; }
CMTV_NO_ZC_IN=1 timeout -k 10 300 python bench.py $Q > "$OUT/bench_nofuse.json" 2> "$OUT/bench_nofuse.err" || { tail -20 "$OUT/bench_nofuse.err"; exit 1; }
python - <<'PY'
import json
for f in ("fused", "nofuse"):
    d = json.load(open(f"gpurun_out/fuse/bench_{f}.json"))
    print(f, d["value"], d["latency_150"]["p50_ms"], d["latency_150"]["p99_ms"], d["latency_150"]["keyset_cache"]["p50_ms"], d.get("replay_150", {}).get("ms_per_height_plain"))
PY
