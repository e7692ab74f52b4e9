#!/bin/bash
# r03: the fused kernel (bit-identical unit tests, timing, timelines) and the split-K order, then a
# step A/B of the fused kernel per tower (MAPFED_FUSED_QKV_ATTN) and the split-K order.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "qkv_attention or splitk or fused" \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; echo "unit rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_fused.log | tail -5
[ $rc -eq 0 ] || exit $rc
bash scripts/qkv_stamps.sh > gpurun_out/qkv_stamps_run.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep -E "occupancy|qkv_attn|gemm |peak" gpurun_out/qkv_stamps.log
[ $rc -eq 0 ] || exit $rc
for wv in 14; do
  MAPFED_QKV_WAVES=$wv timeout -k 10 180 python -u tests/diagnostics/qkv_attn_bench.py > gpurun_out/qkv_attn_bench_w$wv.txt 2>&1
  rc=$?; echo "qkv bench waves=$wv rc=$rc"; grep -v Warn gpurun_out/qkv_attn_bench_w$wv.txt | grep -v amdgpu.ids
  [ $rc -eq 0 ] || exit $rc
done
VARIANTS="${VARIANTS:-MAPFED_FUSED_QKV_ATTN=0 MAPFED_FUSED_QKV_ATTN=text MAPFED_FUSED_QKV_ATTN=1 MAPFED_SPLITK_ORDER=0}" \
  ROUNDS=${ROUNDS:-2} BENCH_ARGS="--no-c5 --no-caption-mode" bash scripts/bench_ab.sh
