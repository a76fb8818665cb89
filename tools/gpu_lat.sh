set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lat
timeout -k 10 120 python tools/commit_phases.py --n 150 --iters 1000 > gpurun_out/lat/phases.log 2>&1 || { tail -20 gpurun_out/lat/phases.log; exit 1; }
grep -v amdgpu.ids gpurun_out/lat/phases.log
timeout -k 10 180 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d gpurun_out/lat/trace -o run -- python3 tools/lat_probe.py 300 > gpurun_out/lat/probe.log 2>&1 || { tail -20 gpurun_out/lat/probe.log; exit 1; }
tail -3 gpurun_out/lat/probe.log
d=$(dirname $(find gpurun_out/lat/trace -name 'run_hip_api_trace.csv' | head -1))
python3 tools/lat_timeline.py $d 200 > gpurun_out/lat/timeline.txt 2>&1; tail -40 gpurun_out/lat/timeline.txt
