#!/bin/bash
# round 6: keyed 10k commit reading its signatures in place (CMTV_KEYED_ZC=1,
# no early DMA) vs the early DMA, three alternating rounds
set -o pipefail
OUT=gpurun_out/r6x
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2 3; do
  for Z in 1 0; do
    CMTV_KEYED_ZC=$Z timeout -k 10 200 python -u tools/vc10k_ab.py 300 > "$OUT/zc${Z}_r$R.json" 2> "$OUT/zc${Z}_r$R.err" || { tail "$OUT/zc${Z}_r$R.err"; exit 1; }
    echo "keyed_zc=$Z round $R $(tail -1 "$OUT/zc${Z}_r$R.json")"
  done
done
