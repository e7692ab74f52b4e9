#!/bin/bash
# r03: check the fused in-projection + attention kernel alone first (unit test + timing), then the full
# session (scripts/gpu_r03.sh).  Any failing GPU step ends the call.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -k "qkv_attention" -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "fused unit rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_fused.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tests/diagnostics/qkv_attn_bench.py > gpurun_out/qkv_attn_bench.txt 2>&1
rc=$?; echo "qkv bench rc=$rc"; cat gpurun_out/qkv_attn_bench.txt | grep -v Warn
[ $rc -eq 0 ] || exit $rc
exec_rc=0
bash scripts/gpu_r03.sh || exec_rc=$?
exit $exec_rc
