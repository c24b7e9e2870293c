#!/bin/bash
# A/B of two builds of the library on the GEMM probe shapes, alternating processes on one box:
#   scripts/ab_gemm.sh <variant.so> [script args]   (B = the in-tree libboxfusion_hip.so)
V=$1; shift
for r in 1 2; do
  echo "== A ($V)"; BF_LIB_PATH=$V timeout -k 10 200 python -u scripts/gemm_tile_sweep.py --auto-only "$@" || exit 1
  echo "== B (in-tree)"; timeout -k 10 200 python -u scripts/gemm_tile_sweep.py --auto-only "$@" || exit 1
done
