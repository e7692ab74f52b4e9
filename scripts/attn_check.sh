#!/bin/bash
# Attention-only GPU session: numerics (default variants), then fwd/bwd timing per variant pair.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for kt in 1 2; do MAPFED_ATTN_BWD_KT=$kt MAPFED_ATTN_FWD=$((kt == 1 ? 4 : 1)) timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "pytest (bwd KT=$kt) rc=$rc"; tail -3 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit $rc; done
for v in ${VARIANTS:-1:1:1 1:2:1}; do
  IFS=: read -r vf vb vk vn <<< "$v"
  MAPFED_ATTN_FWD=$vf MAPFED_ATTN_BWD=$vb MAPFED_ATTN_BWD_KT=${vk:-1} MAPFED_ATTN_FWD_NW=${vn:-4} timeout -k 10 200 python -u tests/diagnostics/attn_bench.py > gpurun_out/attn_bench.log 2>&1
  rc=$?; echo "fwd:bwd variant $v rc=$rc"; cat gpurun_out/attn_bench.log; [ $rc -eq 0 ] || exit $rc
done
