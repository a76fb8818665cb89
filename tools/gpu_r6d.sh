#!/bin/bash
# round 6: rocprof evidence of this round's bench (TAG=r06) + host phases of the 10k keyset commit
set -o pipefail
mkdir -p gpurun_out/r6d
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/vc10k_phases.py 300 > gpurun_out/r6d/vc10k_phases.txt 2>&1 || exit 1
cat gpurun_out/r6d/vc10k_phases.txt | grep -v amdgpu.ids
TAG=r06 bash tools/gpu_prof_r04.sh
