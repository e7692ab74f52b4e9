#!/bin/bash
# Attention forward variants A/B (isolated kernel timing + output checksums).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/attn_variants.log
# VARIANTS: space-separated env assignments per run, e.g. "MAPFED_ATTN_LSUM=0 MAPFED_ATTN_LSUM=1"
for v in ${VARIANTS:-MAPFED_ATTN_FWD=4 MAPFED_ATTN_FWD=1}; do
  echo "== $v" >> gpurun_out/attn_variants.log
  env "$v" timeout -k 10 120 python -u tests/diagnostics/attn_bench.py >> gpurun_out/attn_variants.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc at $v"; cat gpurun_out/attn_variants.log; exit $rc; }
done
cat gpurun_out/attn_variants.log
