#!/bin/bash
# r03: the LDS-occupancy probe (how many workgroups the dispatcher co-locates per CU by LDS size and block
# size), then the GPU test tier with parity reports (including the four extra C4 B=32 eval fixtures).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 tests/diagnostics/lds_occupancy.cpp -o gpurun_out/lds_occ 2> gpurun_out/lds_occ_build.log
rc=$?; [ $rc -eq 0 ] || { echo "build rc=$rc"; tail gpurun_out/lds_occ_build.log; exit $rc; }
timeout -k 10 120 gpurun_out/lds_occ > gpurun_out/lds_occ.log 2>&1
rc=$?; echo "lds_occ rc=$rc"; cat gpurun_out/lds_occ.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/parity
DIST=0 BENCH=0 bash scripts/gpu_r03.sh
timeout -k 10 300 python -u tests/diagnostics/ln_bound_probe.py > gpurun_out/ln_bound_probe.txt 2>&1
rc=$?; echo "ln probe rc=$rc"; grep -E "ms/step|Error" gpurun_out/ln_bound_probe.txt
