#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace. Stops at the first fault.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
fi
exit 0
