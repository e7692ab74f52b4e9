#!/bin/bash
# r03: persistent 256x256 GEMM, 16-byte register epilogue (tile 27: next prologue before the epilogue, 28: after):
# bit-identity tests, C5 shapes, per-tile stamps.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "persistent" -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_j.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/diagnostics/gemm_bench.py 20,27,28 c5 > gpurun_out/gemm_bench_c5.txt 2>&1
rc=$?; echo "gemm bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench_c5.txt
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/gemm_stamps.txt
SHAPES="77000 2048 512 3 20;77000 2048 512 3 27;77000 2048 512 3 28;77000 2048 512 4 27;77000 512 512 2 27" bash scripts/gemm_stamps.sh
