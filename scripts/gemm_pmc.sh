#!/bin/bash
# PMC passes over ONE GEMM configuration (args: M N K epilogue tile), one counter group per run.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="$*"
TAG=$(echo "$ARGS" | tr ' ' '_')
P="python3 tests/diagnostics/gemm_one.py $ARGS 10"
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace -f csv -d gpurun_out/gpmc_${TAG}_$i -o run -- $P > gpurun_out/gpmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/gpmc_${TAG}_$i.log; exit $rc; }
done
python3 - "$TAG" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"gpurun_out/gpmc_{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm" not in r["Kernel_Name"]: continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
disp = None
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:16.0f}  per-dispatch-row-avg {tot[k]/max(n[k],1):14.1f}  rows {n[k]}")
PY
