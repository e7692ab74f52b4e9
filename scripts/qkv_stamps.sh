#!/bin/bash
# In-kernel phase timelines of the fused in-projection + attention forward (tests/diagnostics/qkv_stamps.cpp),
# built on the box; vision c4 shape and the text shapes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
hipcc -O3 -std=c++17 --offload-arch=gfx950 tests/diagnostics/qkv_stamps.cpp -o gpurun_out/qkv_stamps 2> gpurun_out/qkv_stamps_build.log
rc=$?; [ $rc -eq 0 ] || { echo "build rc=$rc"; tail gpurun_out/qkv_stamps_build.log; exit $rc; }
: > gpurun_out/qkv_stamps.log
for shape in "32 199 12 0" "38 77 8 1" "1000 77 8 1"; do
  timeout -k 10 60 gpurun_out/qkv_stamps $shape >> gpurun_out/qkv_stamps.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc at $shape"; cat gpurun_out/qkv_stamps.log; exit $rc; }
done
cat gpurun_out/qkv_stamps.log
