#!/bin/bash
# Bit-identity A/B: tests/diagnostics/step_digest.py in the repo and in _ab/ (a copy of an earlier commit with
# its own libmapfed.so, made on the CPU side: scripts/make_ab.sh <rev>); equal lines = identical results.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for d in . _ab; do
  (cd $d && timeout -k 10 300 python -u tests/diagnostics/step_digest.py ${DIGEST_CFGS:-c4 c5}) > gpurun_out/digest_$( [ $d = . ] && echo new || echo old ).txt 2> gpurun_out/digest_err.txt
  rc=$?; [ $rc -eq 0 ] || { echo "$d rc=$rc"; tail -5 gpurun_out/digest_err.txt; exit $rc; }
done
echo "old:"; cat gpurun_out/digest_old.txt; echo "new:"; cat gpurun_out/digest_new.txt
cmp -s gpurun_out/digest_old.txt gpurun_out/digest_new.txt && echo "DIGESTS IDENTICAL" || echo "DIGESTS DIFFER"
