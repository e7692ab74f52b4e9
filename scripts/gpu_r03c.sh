#!/bin/bash
# r03 measurement session: fused-kernel timelines (qkv_stamps.sh), the GPU test tier with the floor-relative
# parity gates (parity reports under gpurun_out/parity), the default bench line, and rocprofv3 kernel-trace
# summaries of a short c4 bench and a short c5 bench.  Every GPU step has its own time limit; a step that
# crashes ends the session.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${STAMPS:-1}" = "1" ]; then
  bash scripts/qkv_stamps.sh > gpurun_out/qkv_stamps_run.log 2>&1
  rc=$?; echo "stamps rc=$rc"; grep -E "occupancy|qkv_attn|gemm |peak" gpurun_out/qkv_stamps.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SPLITK:-1}" = "1" ]; then
  for o in 0 1 0 1; do
    MAPFED_SPLITK_ORDER=$o timeout -k 10 120 python -u tests/diagnostics/splitk_bench.py >> gpurun_out/splitk_ab.log 2>&1
    rc=$?; echo "splitk order=$o rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  cat gpurun_out/splitk_ab.log
fi
DIST=0 bash scripts/gpu_r03.sh || exit $?
if [ "${PROFILE:-1}" = "1" ]; then
  for cfg in c4 c5; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_$cfg -o run -- \
      python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-eot-mode --no-c5 --no-caption-mode \
      > gpurun_out/prof_$cfg.log 2>&1
    rc=$?; echo "rocprof $cfg rc=$rc"; tail -1 gpurun_out/prof_$cfg.log | cut -c1-300
    [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
