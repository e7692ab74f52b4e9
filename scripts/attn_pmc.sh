#!/bin/bash
# PMC passes over the attention kernels on the c4 shapes (tests/diagnostics/attn_pmc_run.py, eager launches),
# one counter group per run, summarised per kernel by tests/diagnostics/attn_pmc_summary.py.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
dirs=""
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "attn_" -f csv -d gpurun_out/apmc_$i -o run \
    -- python3 tests/diagnostics/attn_pmc_run.py > gpurun_out/apmc_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/apmc_$i.log; exit $rc; }
  dirs="$dirs gpurun_out/apmc_$i"
done
python3 tests/diagnostics/attn_pmc_summary.py gpurun_out/attn_pmc_summary.json $dirs
