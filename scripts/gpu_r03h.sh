#!/bin/bash
# r03: dimg kernel (one wave per row x 64-column chunk) and the caption-pool vocab bound: head / caption kernel
# tests, bit-identity digest A/B against _ab/ (HEAD before the change), then the PMC passes of the c4 bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_captions_gpu.py -k "head or caption_kernels" \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_h.log | tail -4
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_digest.sh || exit $?
bash scripts/gemm_stamps.sh || exit $?
[ "${PMC:-1}" = "1" ] || exit 0
BENCH_ARGS="--no-c5 --no-eot-mode --no-caption-mode" bash scripts/gpu_pmc.sh
