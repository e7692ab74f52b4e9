#!/bin/bash
# Attention launch-shape sweep (fwd4 waves per workgroup x query split), isolated kernel timing.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/attn_sweep.log
for cfg in ${CFGS:-0:0 4:2 5:2 7:2 4:3 4:1 8:1 13:1}; do
  IFS=: read -r w qs <<< "$cfg"
  echo "== waves=$w qsplit=$qs" >> gpurun_out/attn_sweep.log
  MAPFED_ATTN_FWD_WAVES=$w MAPFED_ATTN_QSPLIT=$qs timeout -k 10 120 python -u tests/diagnostics/attn_bench.py >> gpurun_out/attn_sweep.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc at $cfg"; exit $rc; }
done
cat gpurun_out/attn_sweep.log
