#!/bin/bash
# r03: text-tower tile A/B in the c4 step (bigger text tiles = fewer CU-seconds beside the vision tower?)
set -u
cd "$(dirname "$0")/.."
VARIANTS="${VARIANTS:-- MAPFED_TEXT_TILE=10 MAPFED_TEXT_TILE=10,MAPFED_TEXT_LIB=0 MAPFED_TEXT_TILE=11 MAPFED_TEXT_TILE=16}" ROUNDS=2 BENCH_STEPS=20 \
  BENCH_ARGS="--no-c5 --no-caption-mode" bash scripts/bench_ab.sh
