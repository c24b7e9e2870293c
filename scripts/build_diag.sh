#!/bin/bash
# Diagnostic build of libboxfusion_hip.so that routes every call through the rare / generic
# kernel paths (hull IoU with > 4 candidates on the scratch path, NMS scan without the
# single-wave LDS variant, one workgroup per OBB pair, one launch per refinement iteration).  The GPU tests run against it with
#   BF_LIB_PATH=boxfusion_amd/_build/diag/libboxfusion_hip_diag.so pytest tests/test_gpu_fusion.py
# to show that those paths give the same results as the fast ones.
set -e
cd "$(dirname "$0")/../boxfusion_amd/_build"
python3 -c "import sys; sys.path.insert(0, '../..'); from boxfusion_amd import build; build.build()"
mkdir -p diag
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I../../include -Wno-unused-result"
/opt/rocm/bin/hipcc $FL -DFAST_CAND=4 -DFUSE_SPLIT_ITER=0 -c ../csrc/bf_fusion.hip -o diag/bf_fusion.o
/opt/rocm/bin/hipcc $FL -DNMS_FAST_N=0 -c ../csrc/bf_assoc.hip -o diag/bf_assoc.o
/opt/rocm/bin/hipcc $FL -DOBB_SPLIT=0 -DOBB_LAST_BLOCK=1 -c ../csrc/bf_iou3d.hip -o diag/bf_iou3d.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o diag/libboxfusion_hip_diag.so \
    $(ls *.o | grep -v -e "^bf_fusion.o$" -e "^bf_assoc.o$" -e "^bf_iou3d.o$") diag/bf_fusion.o diag/bf_assoc.o diag/bf_iou3d.o
echo "$PWD/diag/libboxfusion_hip_diag.so"
