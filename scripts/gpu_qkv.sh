#!/bin/bash
# the fused in-projection + attention kernel: unit tests (bit-identical to the unfused pair) then timing
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -k "qkv_attention" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "fused unit rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_fused.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tests/diagnostics/qkv_attn_bench.py > gpurun_out/qkv_attn_bench.txt 2>&1
rc=$?; echo "qkv bench rc=$rc"; grep -v Warn gpurun_out/qkv_attn_bench.txt | grep -v amdgpu.ids
exit $rc
