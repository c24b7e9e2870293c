#!/bin/bash
# A/B variant of libboxfusion_hip.so: the given -D flags on the fusion-side sources, into
# boxfusion_amd/_build/variant/libboxfusion_hip_variant.so (run with BF_LIB_PATH=...).
set -e
cd "$(dirname "$0")/../boxfusion_amd/_build"
python3 -c "import sys; sys.path.insert(0, '../..'); from boxfusion_amd import build; build.build()"
mkdir -p variant
FL="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I../../include -Wno-unused-result"
for f in bf_fusion bf_assoc bf_iou3d; do /opt/rocm/bin/hipcc $FL "$@" -c ../csrc/$f.hip -o variant/$f.o; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variant/libboxfusion_hip_variant.so \
    $(ls *.o | grep -v -e "^bf_fusion.o$" -e "^bf_assoc.o$" -e "^bf_iou3d.o$") variant/bf_fusion.o variant/bf_assoc.o variant/bf_iou3d.o
echo "$PWD/variant/libboxfusion_hip_variant.so"
