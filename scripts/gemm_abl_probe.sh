#!/bin/bash
# GEMM K-loop ablations (diagnostic builds, wrong results): in-tree lib vs GEMM_ABL=1 (no LDS-DMA
# in the K loop), 2 (no fragment reads), 3 (neither), each on real and on L2-resident operands
# (scripts/gemm_l2_probe.py), alternating processes on one box.
for r in 1 2; do
  echo "== full"; timeout -k 10 120 python -u scripts/gemm_l2_probe.py || exit 1
  for v in 1 2 3; do echo "== abl $v"; BF_LIB_PATH=boxfusion_amd/_build/variant/lib_abl$v.so timeout -k 10 120 python -u scripts/gemm_l2_probe.py || exit 1; done
done
