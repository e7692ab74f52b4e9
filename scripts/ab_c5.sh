#!/bin/bash
# Interleaved A/B of bench.py engine options on the C5 step (bench.py --config c5, K = 1 000 classes): VARIANTS
# as in bench_ab.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:--}; do
    vargs=""; [ "$v" != "-" ] && vargs="${v//,/ }"
    out=$(timeout -k 10 300 python bench.py $vargs --config c5 --steps ${BENCH_STEPS:-10} --warmup 2 --no-cpu-baseline \
          --no-eot-mode --no-round --no-c5 --no-caption-mode 2> gpurun_out/ab_c5.err)
    rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -3 gpurun_out/ab_c5.err; exit $rc; }
    echo "$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "img/s", round(d["ms_per_step"],3), "ms")')"
  done
done
