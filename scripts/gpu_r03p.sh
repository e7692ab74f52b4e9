#!/bin/bash
# r03: text-tower LayerNorm rows per half-wave and text attention query split: bit-identity (step digests with
# each knob against none), then the c4 step A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in - MAPFED_LN_TEXT_RPH=2 MAPFED_LN_TEXT_RPH=4 MAPFED_ATTN_QSPLIT_TEXT=1 MAPFED_ATTN_QSPLIT_TEXT=3; do
  envs=""; [ "$v" != "-" ] && envs="$v"
  env $envs timeout -k 10 300 python -u tests/diagnostics/step_digest.py c4 > gpurun_out/dig_$v.txt 2> gpurun_out/dig_err.txt
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/dig_err.txt; exit $rc; }
  echo "$v $(cat gpurun_out/dig_$v.txt)"
done
VARIANTS="- MAPFED_LN_TEXT_RPH=2 MAPFED_LN_TEXT_RPH=4 MAPFED_ATTN_QSPLIT_TEXT=1 MAPFED_ATTN_QSPLIT_TEXT=3" ROUNDS=2 \
  BENCH_STEPS=20 BENCH_ARGS="--no-c5 --no-caption-mode" bash scripts/bench_ab.sh
