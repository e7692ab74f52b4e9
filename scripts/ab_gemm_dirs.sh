#!/bin/bash
# GEMM A/B of two trees on one box, interleaved (tests/diagnostics/gemm_bench.py, heuristic tiles, c4 shapes):
# the repo (.) against a copy under _ab/ (git-ignored, deleted after use); then the bench A/B (ab_dirs.sh).
set -u
cd "$(dirname "$0")/.."
for r in $(seq 1 ${ROUNDS:-2}); do
  for d in . _ab; do
    echo "== $d round $r"
    (cd $d && timeout -k 10 200 python -u tests/diagnostics/gemm_bench.py 0) 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "$d rc=$rc"; exit $rc; }
  done
done
[ "${BENCH_AB:-1}" = "1" ] && ROUNDS=${BENCH_ROUNDS:-2} bash scripts/ab_dirs.sh
