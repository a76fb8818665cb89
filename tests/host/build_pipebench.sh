#!/bin/bash
# Builds tests/host/pipebench (host cost of the cross-height pipeline over
# fake devices; no GPU, no sanitizers). Usage: tests/host/build_pipebench.sh
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OBJ=$ROOT/build/pipebench
mkdir -p "$OBJ"
# the library's own compiler and flags for the code under test (hipcc
# host compile, cometbft_amd/csrc/Makefile CXXFLAGS), g++ for the harness
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
for f in cometbft_amd/csrc/commit.cpp cometbft_amd/csrc/pipeline.cpp; do
  $HIPCC -O3 -std=c++17 -fPIC -c "$ROOT/$f" -o "$OBJ/$(basename "$f").o" &
done
FL="-O2 -g -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include"
for f in tests/host/pipebench.cpp tests/host/fake_runtime.cpp; do
  g++ $FL -c "$ROOT/$f" -o "$OBJ/$(basename "$f").o" &
done
gcc -O2 -c "$ROOT/oracle/cmtv_oracle.c" -o "$OBJ/oracle.o" &
wait
g++ -o "$ROOT/tests/host/pipebench" "$OBJ"/*.o -lpthread -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
