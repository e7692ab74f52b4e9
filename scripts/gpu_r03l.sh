#!/bin/bash
# r03: kept persistent variant (tile 27) on the C5 in-projection: tests, heuristic C5 shapes, C5 step digests vs _ab/
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "persistent or gemm_bias" -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_l.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_l.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/diagnostics/gemm_bench.py 0,20,10 c5 > gpurun_out/gemm_bench_c5.txt 2>&1
rc=$?; echo "gemm bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench_c5.txt
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c5 c4" bash scripts/ab_digest.sh
