#!/bin/bash
# Attention forward variants A/B (isolated kernel timing + output checksums).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/attn_variants.log
for v in ${VARIANTS:-4 5}; do
  echo "== MAPFED_ATTN_FWD=$v" >> gpurun_out/attn_variants.log
  MAPFED_ATTN_FWD=$v timeout -k 10 120 python -u tests/diagnostics/attn_bench.py >> gpurun_out/attn_variants.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc at $v"; cat gpurun_out/attn_variants.log; exit $rc; }
done
cat gpurun_out/attn_variants.log
