#!/bin/bash
# One GPU-box session made of named steps, run in the order given; each GPU step has its own time limit and the
# first failing step ends the session (nothing further touches the GPU).  Outputs go under gpurun_out/.
#
#   gpurun --timeout 1200 -- bash scripts/gpu.sh tests bench prof
#
# steps (knobs are environment variables):
#   tests      pytest -m gpu, parity reports under gpurun_out/parity   (PYTEST_ARGS, TEST_TIMEOUT)
#   sel        pytest on the files / node ids in SEL                    (PYTEST_ARGS)
#   bench      the default bench line, CPU baseline included            (BENCH_ARGS, BENCH_STEPS)
#   quick      a bench line without the CPU baseline, round wall-time, caption and EOT side runs (BENCH_ARGS)
#   prof       rocprofv3 --kernel-trace --stats of a 5-step c4 bench -> gpurun_out/prof  (BENCH_ARGS)
#   profc5     the same for the C5 side config (bench.py --config c5)
#   pmc_gemm   FETCH_SIZE / WRITE_SIZE passes over tests/diagnostics/gemm_traffic.py -> gpurun_out/gemm_traffic.json
#   gemm       tests/diagnostics/gemm_bench.py $GEMM_TILES $GEMM_SET   (tile A/B per shape against hipBLASLt)
#   digest     tests/diagnostics/step_digest.py $DIGEST_CFGS (bit-identity A/B of two trees: compare the lines)
#   ab         interleaved bench A/B of bench.py options: VARIANTS="--text-first -" ROUNDS times (scripts/bench_ab.sh)
#   attn       tests/diagnostics/attn_bench.py $ATTN_ARGS
#   pmc_bench  FETCH / WRITE / MFMA-busy passes over a short bench run (scripts/gpu_pmc.sh -> gpurun_out/pmc_summary.json)
#   pmc_attn   PMC passes over the attention kernels (scripts/attn_pmc.sh -> gpurun_out/attn_pmc_summary.json)
#   pmc_probe  stall / LDS / MFMA counter passes over single GEMM launches (scripts/gemm_pmc_probe.sh; CONFIGS, LIB)
#   stamps_gemm / stamps_attn / stamps_qkv   in-kernel timelines (scripts/{gemm,attn,qkv}_stamps.sh; SHAPES)
#   ab_c5      interleaved C5 A/B of bench.py options (scripts/ab_c5.sh; VARIANTS, ROUNDS)
# Two-tree A/B (scripts/make_ab.sh REV, then scripts/ab_dirs.sh / ab_digest.sh) and ab_gemm_dirs.sh stay separate:
# they need a second build of the library prepared on the CPU side first.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
QUICK="--no-cpu-baseline --no-round --no-eot-mode --no-c5 --no-caption-mode --no-eval"

step() {
  case "$1" in
    tests)
      MAPFED_PARITY_REPORT=gpurun_out/parity timeout -k 10 ${TEST_TIMEOUT:-1200} python -u -m pytest tests -m gpu -v -s \
        --maxfail=10 --timeout 420 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_gpu.log | tail -12
      return $rc ;;
    sel)
      timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${SEL} -v -s --timeout 420 --timeout-method thread \
        ${PYTEST_ARGS:-} > gpurun_out/pytest_sel.log 2>&1
      rc=$?; echo "sel rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_sel.log | tail -12
      return $rc ;;
    bench)
      timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py --steps ${BENCH_STEPS:-20} --warmup 5 ${BENCH_ARGS:-} \
        > gpurun_out/bench.json 2> gpurun_out/bench.err
      rc=$?; echo "bench rc=$rc"; cut -c1-700 gpurun_out/bench.json; tail -3 gpurun_out/bench.err
      return $rc ;;
    quick)
      timeout -k 10 300 python -u bench.py --steps ${BENCH_STEPS:-20} --warmup 3 $QUICK ${BENCH_ARGS:-} \
        > gpurun_out/quick.json 2> gpurun_out/quick.err
      rc=$?; echo "quick rc=$rc"; python3 -c 'import json;d=json.load(open("gpurun_out/quick.json"));r=d["roofline"];print(round(d["value"],1),"img/s",round(d["ms_per_step"],3),"ms; gemm frac",round(r["frac"],4),"avg",round(r["avg_launch_us"],2),"us")'
      return $rc ;;
    prof|profc5)
      local cfg=""; [ "$1" = "profc5" ] && cfg="--config c5"
      timeout -k 10 ${PROF_TIMEOUT:-500} rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$1 -o run -- \
        python3 bench.py --steps 5 --warmup 1 $QUICK $cfg ${BENCH_ARGS:-} > gpurun_out/$1.log 2>&1
      rc=$?; echo "$1 rc=$rc"; tail -2 gpurun_out/$1.log
      return $rc ;;
    pmc_gemm)
      rm -rf gpurun_out/gt_fetch gpurun_out/gt_write
      for ctr in FETCH_SIZE WRITE_SIZE; do
        local d=gpurun_out/gt_$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
        timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -f csv -d $d -o run -- \
          python3 tests/diagnostics/gemm_traffic.py run gpurun_out/gt_probe.json > $d.log 2>&1
        rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || { tail -5 $d.log; return $rc; }
      done
      python3 tests/diagnostics/gemm_traffic.py summarize gpurun_out/gt_probe.json \
        $(ls gpurun_out/gt_fetch/*counter_collection.csv | head -1) $(ls gpurun_out/gt_write/*counter_collection.csv | head -1) \
        gpurun_out/gemm_traffic.json > gpurun_out/gemm_traffic.txt 2>&1
      rc=$?; echo "pmc summary rc=$rc"; head -3 gpurun_out/gemm_traffic.txt
      return $rc ;;
    gemm)
      timeout -k 10 ${GEMM_TIMEOUT:-400} python3 -u tests/diagnostics/gemm_bench.py ${GEMM_TILES:-0} ${GEMM_SET:-} \
        > gpurun_out/gemm_bench.txt 2>&1
      rc=$?; echo "gemm rc=$rc"; cat gpurun_out/gemm_bench.txt | grep -v amdgpu.ids
      return $rc ;;
    digest)
      timeout -k 10 300 python3 -u tests/diagnostics/step_digest.py ${DIGEST_CFGS:-c4 c5} > gpurun_out/digest.txt 2>&1
      rc=$?; echo "digest rc=$rc"; grep -v amdgpu.ids gpurun_out/digest.txt
      return $rc ;;
    ab)
      bash scripts/bench_ab.sh
      return $? ;;
    attn)
      timeout -k 10 300 python3 -u tests/diagnostics/attn_bench.py ${ATTN_ARGS:-} > gpurun_out/attn_bench.txt 2>&1
      rc=$?; echo "attn rc=$rc"; grep -v amdgpu.ids gpurun_out/attn_bench.txt | tail -40
      return $rc ;;
    pmc_bench)  # the per-dispatch CSVs are large: only the summary is kept
      BENCH_ARGS="$QUICK ${BENCH_ARGS:-}" bash scripts/gpu_pmc.sh; rc=$?
      rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_mfma; return $rc ;;
    pmc_attn) bash scripts/attn_pmc.sh; rc=$?; rm -rf gpurun_out/apmc_*/; return $rc ;;
    pmc_probe) bash scripts/gemm_pmc_probe.sh; return $? ;;
    stamps_gemm) bash scripts/gemm_stamps.sh; return $? ;;
    stamps_attn) bash scripts/attn_stamps.sh; return $? ;;
    stamps_qkv) bash scripts/qkv_stamps.sh; return $? ;;
    ab_c5) bash scripts/ab_c5.sh; return $? ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}

for s in "$@"; do
  step "$s" || exit $?
done
exit 0
