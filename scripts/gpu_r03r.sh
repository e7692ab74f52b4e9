#!/bin/bash
# r03: explicit side-tower tile hint (tile -1): digests vs _ab/ (c4, c5), c4 and C5 step A/B (MAPFED_SIDE_TILES=0)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_r.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_r.log | tail -3
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c4 c5" bash scripts/ab_digest.sh || exit $?
VARIANTS="- MAPFED_SIDE_TILES=0" ROUNDS=2 BENCH_STEPS=20 BENCH_ARGS="--no-c5 --no-caption-mode" bash scripts/bench_ab.sh || exit $?
VARIANTS="- MAPFED_SIDE_TILES=0" ROUNDS=2 BENCH_STEPS=5 BENCH_ARGS="--config c5 --no-c5 --no-caption-mode" bash scripts/bench_ab.sh
