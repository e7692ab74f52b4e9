#!/bin/bash
# Attention-only GPU session: numerics, then fwd/bwd timing for the old (1) and new (2) forward.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-1 2}; do
  MAPFED_ATTN_FWD=$v timeout -k 10 200 python -u tests/diagnostics/attn_bench.py > gpurun_out/attn_bench_$v.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; cat gpurun_out/attn_bench_$v.log; [ $rc -eq 0 ] || exit $rc
done
