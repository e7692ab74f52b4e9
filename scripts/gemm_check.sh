#!/bin/bash
# GEMM-only GPU session: numerics of every tile family, then the shape sweep vs hipBLASLt.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k gemm -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/diagnostics/gemm_bench.py ${TILES:-0,20,21,22,23,24} > gpurun_out/gemm_bench.log 2>&1
rc=$?; cat gpurun_out/gemm_bench.log; exit $rc
