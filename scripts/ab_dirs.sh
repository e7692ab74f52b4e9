#!/bin/bash
# A/B of two trees on one box, interleaved: the repo (.) against a copy under _ab/ (e.g. the package
# from an earlier commit with the same libmapfed.so; _ab/ is git-ignored and deleted after use).
set -u
cd "$(dirname "$0")/.."
for r in $(seq 1 ${ROUNDS:-3}); do
  for d in . _ab; do
    out=$(cd $d && timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --no-cpu-baseline --no-eot-mode 2>/dev/null)
    rc=$?; [ $rc -eq 0 ] || { echo "$d rc=$rc"; exit $rc; }
    echo "$d $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1))')"
  done
done
