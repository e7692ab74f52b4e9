#!/bin/bash
# r03: persistent 256x256 GEMM (tile 27) for the C5 text products: bit-identity tests against gemm8s, the
# C5 GEMM shapes (tiles 20 / 27 / 10), step digests against _ab/, then the C5 step A/B (MAPFED_GEMM_PERSIST=0).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_i.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_i.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/diagnostics/gemm_bench.py 20,27,10 c5 > gpurun_out/gemm_bench_c5.txt 2>&1
rc=$?; echo "gemm bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench_c5.txt
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c5" bash scripts/ab_digest.sh || exit $?
VARIANTS="- MAPFED_GEMM_PERSIST=0" ROUNDS=2 BENCH_STEPS=5 BENCH_ARGS="--config c5 --no-c5 --no-caption-mode" bash scripts/bench_ab.sh
