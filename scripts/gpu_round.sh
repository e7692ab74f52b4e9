#!/bin/bash
# One GPU-box session: the GPU test tier (parity reports under gpurun_out/parity), the default bench line
# (CPU baseline included), and a rocprofv3 kernel-trace summary of a short bench.  Every GPU step has its
# own time limit; the first failing step ends the session (nothing further touches the GPU).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  MAPFED_PARITY_REPORT=gpurun_out/parity timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -v -s \
    --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ${BENCH_ARGS:-} \
    > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-eot-mode --no-c5 --no-caption-mode ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof.log
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
