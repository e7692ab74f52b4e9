#!/bin/bash
# In-kernel GEMM timelines (tests/diagnostics/gemm_stamps.cpp): per-workgroup prologue / main loop / epilogue
# and the start-time histogram, for the shapes in $SHAPES ("M N K epi tile" separated by ';').
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
(cd tests/diagnostics && hipcc -O3 -std=c++17 --offload-arch=gfx950 -DMF_GEMM_STAMPS \
  -I../../federated_multi_modal_amd/csrc gemm_stamps.cpp -o ../../gpurun_out/gemm_stamps) > gpurun_out/gemm_stamps_build.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "stamps build rc=$rc"; tail -5 gpurun_out/gemm_stamps_build.log; exit $rc; }
IFS=';' read -ra SH <<< "${SHAPES:-77000 2048 512 3 20;77000 2048 512 4 20;6368 2304 768 1 20}"
for s in "${SH[@]}"; do
  timeout -k 10 60 gpurun_out/gemm_stamps $s >> gpurun_out/gemm_stamps.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "stamps rc=$rc ($s)"; tail -3 gpurun_out/gemm_stamps.txt; exit $rc; }
done
cat gpurun_out/gemm_stamps.txt
