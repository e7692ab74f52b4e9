#!/bin/bash
# hipBLASLt's kernel (rocprofv3 kernel name: macro tile, depth, stream-K ...) for a few products, via torch.mm in
# tests/diagnostics/gemm_one.py (tile -2).  SHAPES="M,N,K ..."
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/blas_names
for s in ${SHAPES:-19900,2304,768 6368,2304,768}; do
  IFS=, read -r M N K <<< "$s"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/blas_names/${M}_${N}_${K} -o run -- \
    python3 tests/diagnostics/gemm_one.py $M $N $K -2 3 > gpurun_out/blas_names/${M}_${N}_${K}.log 2>&1
  rc=$?; echo "$s rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(ls gpurun_out/blas_names/${M}_${N}_${K}/*kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 -c "import csv,sys; [print('  ', r['Name'][:600], r['AverageNs']) for r in csv.DictReader(open('$f'))]"
  rm -rf gpurun_out/blas_names/${M}_${N}_${K}
done
