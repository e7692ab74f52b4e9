#!/bin/bash
# Attention backward A/B: the attention kernel tests, then isolated timings (tests/diagnostics/attn_bench.py)
# for the fused kernel (MAPFED_ATTN_BWD=2) and the split kernel (=3) at several splits.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k attention --timeout 120 --timeout-method thread \
  > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "attention tests rc=$rc"; tail -3 gpurun_out/attn_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/attn_bwd_ab.log
for v in ${VARIANTS:-2:0 3:0 3:1 3:2 3:3}; do
  IFS=: read -r var sp <<< "$v"
  echo "== MAPFED_ATTN_BWD=$var MAPFED_ATTN_BWD_SPLIT=$sp" >> gpurun_out/attn_bwd_ab.log
  MAPFED_ATTN_BWD=$var MAPFED_ATTN_BWD_SPLIT=$sp timeout -k 10 120 python -u tests/diagnostics/attn_bench.py \
    >> gpurun_out/attn_bwd_ab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc at $v"; cat gpurun_out/attn_bwd_ab.log; exit $rc; }
done
cat gpurun_out/attn_bwd_ab.log
