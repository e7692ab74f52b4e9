#!/bin/bash
# In-kernel phase timelines of the attention backward (tests/diagnostics/attn_stamps.cpp), built on the box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
hipcc -O3 -std=c++17 --offload-arch=gfx950 tests/diagnostics/attn_stamps.cpp -o gpurun_out/attn_stamps 2> gpurun_out/attn_stamps_build.log
rc=$?; [ $rc -eq 0 ] || { echo "build rc=$rc"; tail gpurun_out/attn_stamps_build.log; exit $rc; }
: > gpurun_out/attn_stamps.log
for v in ${VARIANTS:-2:1 3:1 3:2}; do
  IFS=: read -r var sp <<< "$v"
  echo "== MAPFED_ATTN_BWD=$var split=$sp" >> gpurun_out/attn_stamps.log
  MAPFED_ATTN_BWD=$var MAPFED_ATTN_BWD_SPLIT=$sp STAMP_SPLIT=$sp timeout -k 10 60 gpurun_out/attn_stamps ${SHAPE:-32 199 12 0} \
    >> gpurun_out/attn_stamps.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc at $v"; cat gpurun_out/attn_stamps.log; exit $rc; }
done
cat gpurun_out/attn_stamps.log
