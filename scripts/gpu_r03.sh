#!/bin/bash
# r03 GPU session: the GPU test tier (parity reports under gpurun_out/parity), the trainer's distributed
# branch with real kernels (two gloo ranks sharing the GPU: 2 clients, then 4 clients = 2 per rank), and
# the default bench line.  Each GPU step has its own time limit; a failing step ends the session.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  MAPFED_PARITY_REPORT=gpurun_out/parity timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v -s \
    --maxfail=10 --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_gpu.log | tail -12
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ "${DIST:-1}" = "1" ]; then
  for n in 2 4; do
    MAPFED_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $((29611 + n)) tests/diagnostics/dist_trainer_check.py --clients $n \
      --out gpurun_out/dist_check_c$n.json > gpurun_out/dist_c$n.log 2>&1
    rc=$?; echo "dist clients=$n rc=$rc"; grep -E '"ok"' gpurun_out/dist_check_c$n.json | tail -1
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ${BENCH_ARGS:-} \
    > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
