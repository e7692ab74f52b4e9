#!/bin/bash
# PMC passes (one counter group per run, --kernel-trace only) for the bench's kernels.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
for pass in fetch:FETCH_SIZE write:WRITE_SIZE mfma:SQ_VALU_MFMA_BUSY_CYCLES,GRBM_GUI_ACTIVE; do
  name=${pass%%:*}; ctr=${pass#*:}
  timeout -k 10 900 rocprofv3 --pmc ${ctr//,/ } --kernel-trace -f csv -d gpurun_out/pmc_$name -o run -- $B > gpurun_out/pmc_$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_$name.log; exit $rc; }
done
python3 tests/diagnostics/pmc_summary.py gpurun_out/pmc_summary.json \
  fetch=$(ls gpurun_out/pmc_fetch/*counter_collection.csv | head -1) \
  write=$(ls gpurun_out/pmc_write/*counter_collection.csv | head -1) \
  mfma=$(ls gpurun_out/pmc_mfma/*counter_collection.csv | head -1)
