#!/bin/bash
# r03: LDS occupancy probe (static-LDS / VGPR variants), LayerNorm step bound (with the stats-scan stand-in),
# the GEMM shapes against hipBLASLt, and the EOT_TRUNCATE trainer test.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 tests/diagnostics/lds_occupancy.cpp -o gpurun_out/lds_occ 2> gpurun_out/lds_occ_build.log
rc=$?; [ $rc -eq 0 ] || { echo "build rc=$rc"; tail gpurun_out/lds_occ_build.log; exit $rc; }
timeout -k 10 120 gpurun_out/lds_occ > gpurun_out/lds_occ.log 2>&1
rc=$?; echo "lds_occ rc=$rc"; grep -E "static|threads  384 LDS  7" gpurun_out/lds_occ.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_trainers_gpu.py -k eot_truncate -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_eot.log 2>&1
rc=$?; echo "eot test rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_eot.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tests/diagnostics/ln_bound_probe.py > gpurun_out/ln_bound_probe.txt 2>&1
rc=$?; echo "ln probe rc=$rc"; grep -E "ms/step|Error" gpurun_out/ln_bound_probe.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/diagnostics/gemm_bench.py 0 > gpurun_out/gemm_bench.txt 2>&1
rc=$?; echo "gemm bench rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_bench.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_modules_gpu.py -x -q -s --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_modules.log 2>&1
rc=$?; echo "modules rc=$rc"; grep -E "rows 0-1|passed|failed" gpurun_out/pytest_modules.log
