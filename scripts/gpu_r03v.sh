#!/bin/bash
# r03: the towers' dX clears moved beside the vision forward: engine / caption / module tests, step digests vs
# _ab/, c4 step A/B against the previous tree (_ab2/)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_captions_gpu.py tests/test_modules_gpu.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_v.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_v.log | tail -3
[ $rc -eq 0 ] || exit $rc
DIGEST_CFGS="c4 c2" bash scripts/ab_digest.sh || exit $?
ROUNDS=3 bash scripts/ab_dirs.sh
