#!/bin/bash
# r03: the side tower's block-11 weight gradients in one pass on 128x128 (no split-K): c4 parity fixtures, then the
# c4 step A/B (MAPFED_TEXT_TILE=-1 restores every latency pick, for reference)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
MAPFED_PARITY_REPORT=gpurun_out/parity_s timeout -k 10 500 python -u -m pytest tests/test_parity_cases_gpu.py tests/test_engine_gpu.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_s.log | tail -3
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c4" bash scripts/ab_digest.sh
ROUNDS=3 bash scripts/ab_dirs.sh
