#!/bin/bash
# A/B of two trees on one box, interleaved (as scripts/ab_dirs.sh), on the c4 step alone: no FedAvg round, C5,
# caption or EOT-truncated side measurements.  Prints value (img/s) and ms per step per run.
set -u
cd "$(dirname "$0")/.."
for r in $(seq 1 ${ROUNDS:-3}); do
  for d in . _ab; do
    out=$(cd $d && timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --no-cpu-baseline \
          --no-eot-mode --no-round --no-c5 --no-caption-mode 2>/dev/null)
    rc=$?; [ $rc -eq 0 ] || { echo "$d rc=$rc"; exit $rc; }
    echo "$d $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],3))')"
  done
done
