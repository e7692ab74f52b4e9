#!/bin/bash
# r03: the training head in one launch (mf_clip_head_loss_small): bit-identity test, step digests vs _ab/,
# and the c4 step A/B (MAPFED_FUSED_HEAD=0: the eight-launch head)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "head or engine or eot or step" -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|Error" gpurun_out/pytest_q.log | tail -5
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c4 c2" bash scripts/ab_digest.sh || exit $?
VARIANTS="- MAPFED_FUSED_HEAD=0" ROUNDS=3 BENCH_STEPS=20 BENCH_ARGS="--no-c5 --no-caption-mode" bash scripts/bench_ab.sh
