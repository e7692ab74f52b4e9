#!/bin/bash
# r03: optimizer step in three launches (mf_optimizer_step): engine / trainer tests (halt semantics), step digests
# vs _ab/, c4 step A/B (MAPFED_FUSED_OPTIM=0)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_trainers_gpu.py tests/test_kernels_gpu.py -k "sgd or clip or engine or nonfinite or halt or step or failed or input" \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_u.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_u.log | tail -3
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c4 c2" bash scripts/ab_digest.sh || exit $?
VARIANTS="- MAPFED_FUSED_OPTIM=0" ROUNDS=3 BENCH_STEPS=20 BENCH_ARGS="--no-c5 --no-caption-mode" bash scripts/bench_ab.sh
