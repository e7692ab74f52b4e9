#!/bin/bash
# A/B of bench.py engine options on the c4 step, interleaved in one box session: VARIANTS="--text-first
# --fused-qkv-attn=none,--text-first -" entries are bench.py arguments ("-" = none; "," joins several); each
# variant runs ROUNDS times.  Kernel variants are A/B'd as two library builds instead (scripts/ab_dirs.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:--}; do
    vargs=""; [ "$v" != "-" ] && vargs="${v//,/ }"
    out=$(timeout -k 10 300 python bench.py $vargs --steps ${BENCH_STEPS:-20} --warmup 3 --no-cpu-baseline \
          --no-eot-mode --no-round --no-c5 --no-caption-mode ${BENCH_ARGS:-} 2> gpurun_out/ab.err)
    rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -3 gpurun_out/ab.err; exit $rc; }
    echo "$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "img/s", round(d["ms_per_step"],3), "ms; gemm", round(d["roofline"]["avg_launch_us"],2), "us", round(d["roofline"]["frac"],4))')"
  done
done
