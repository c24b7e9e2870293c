#!/bin/bash
# GEMM K-loop / epilogue ablations (diagnostic builds, wrong results): in-tree lib vs GEMM_ABL=1 (no
# LDS-DMA in the K loop), 2 (no fragment reads), 3 (neither), 4 (k_gemm256q epilogue stores dropped
# through out-of-range offsets, the counted waits unchanged), each on real and on L2-resident
# operands (scripts/gemm_l2_probe.py), alternating processes on one box.
# Variant libraries (built here, before the GPU call):
#   cd boxfusion_amd && mkdir -p _build/variant && for v in 1 2 3 4; do
#     hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c csrc/bf_gemm.hip -o _build/variant/bf_gemm_abl$v.o -DGEMM_ABL=$v &&
#     hipcc --offload-arch=gfx950 -shared -fPIC -o _build/variant/lib_abl$v.so $(ls _build/*.o | grep -v /bf_gemm.o) _build/variant/bf_gemm_abl$v.o; done
VARIANTS=${VARIANTS:-1 2 3}
for r in 1 2; do
  echo "== full"; timeout -k 10 120 python -u scripts/gemm_l2_probe.py || exit 1
  for v in $VARIANTS; do echo "== abl $v"; BF_LIB_PATH=boxfusion_amd/_build/variant/lib_abl$v.so timeout -k 10 120 python -u scripts/gemm_l2_probe.py || exit 1; done
done
