#!/bin/bash
# r03: out-projection + residual + ln_2 in one launch (rowln.hip): bit-identity test, step digests vs _ab/,
# c4 step A/B (MAPFED_FUSED_LN2=0, MAPFED_ROWLN_BM=32)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "resid_ln" -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_t.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|Error|assert" gpurun_out/pytest_t.log | tail -6
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c4 c5" bash scripts/ab_digest.sh || exit $?
VARIANTS="- MAPFED_FUSED_LN2=0 MAPFED_ROWLN_BM=32" ROUNDS=2 BENCH_STEPS=20 BENCH_ARGS="--no-c5 --no-caption-mode" bash scripts/bench_ab.sh
