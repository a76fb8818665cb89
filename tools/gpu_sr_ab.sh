set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sr_ab
for r in 1 2; do for cfg in "0:" "1:" "1:2" "1:4"; do hs=${cfg%%:*}; pre=${cfg##*:}; 
  env CMTV_QUAD_HS=$hs ${pre:+CMTV_HS_PRE=$pre} timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-light --no-latency > gpurun_out/sr_ab/b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/sr_ab/b.json').read().strip().splitlines()[-1]); print('hs=$hs pre=$pre sr', d['sr25519']['kernel_ms'], d['sr25519']['verdicts_ok'], 'ed', d['roofline']['kernel_ms'])"
done; done
