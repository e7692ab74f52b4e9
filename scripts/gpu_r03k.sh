#!/bin/bash
# r03: persistent 256x256 GEMM with every other workgroup started late (MAPFED_GEMM_PDELAY s_sleep(127) units)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "persistent" -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_k.log | tail -4
[ $rc -eq 0 ] || exit $rc
for d in 0 2 3 4 6; do
  MAPFED_GEMM_PDELAY=$d timeout -k 10 300 python -u tests/diagnostics/gemm_bench.py 20,27,28 c5 > gpurun_out/gemm_bench_c5_d$d.txt 2>&1
  rc=$?; echo "pdelay $d rc=$rc"; grep -E "c5.fc|c5.dfc|c5.qkv|c5.out" gpurun_out/gemm_bench_c5_d$d.txt
  [ $rc -eq 0 ] || exit $rc
done
