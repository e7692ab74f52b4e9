#!/bin/bash
# r03: hipBLASLt route for the plain / bias-only products (csrc/blaslt.hip): unit + engine + parity tests,
# then the step A/B (MAPFED_GEMM_LIB=0 keeps every product on the hand-written kernels).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
MAPFED_PARITY_REPORT=gpurun_out/parity_lib timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py \
  tests/test_engine_gpu.py tests/test_parity_cases_gpu.py tests/test_modules_gpu.py -x -q -s --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_lib.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|rows 0-1" gpurun_out/pytest_lib.log | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
VARIANTS="- MAPFED_GEMM_LIB=0" ROUNDS=3 BENCH_ARGS="--no-c5 --no-caption-mode" bash scripts/bench_ab.sh
