#!/bin/bash
# _ab/: the package, oracle-free scripts and a freshly built libmapfed.so of git revision $1 (CPU side, before a
# gpurun A/B: scripts/ab_dirs.sh, scripts/ab_digest.sh).  _ab/ is git-ignored.
set -eu
cd "$(dirname "$0")/.."
rm -rf _ab && mkdir _ab
git archive "${1:-HEAD}" federated_multi_modal_amd tests/diagnostics bench.py configs | tar -x -C _ab
make -C _ab/federated_multi_modal_amd/csrc -j8 > /dev/null
ls -la _ab/federated_multi_modal_amd/lib/libmapfed.so
