#!/bin/bash
# r03: tower-overlap bound of the c4 step (full / serial / vision only / text only / CU-masked text stream)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tests/diagnostics/tower_bound_probe.py > gpurun_out/tower_bound_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids gpurun_out/tower_bound_probe.txt | tail -12
