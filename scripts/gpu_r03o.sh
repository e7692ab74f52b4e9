#!/bin/bash
# r03: text tower on 160x128 tiles: step digests against _ab/ (old tile rule), GEMM tests, tower-overlap probe
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_o.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_o.log | tail -4
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c4 c2" bash scripts/ab_digest.sh || exit $?
timeout -k 10 300 python -u tests/diagnostics/tower_bound_probe.py > gpurun_out/tower_bound_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids gpurun_out/tower_bound_probe.txt | tail -8
