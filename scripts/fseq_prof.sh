#!/bin/bash
# kernel trace of the native keyframe sequencer alone (30-object scene, 6 steps of 64 keyframes)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
BF_SEQ_OBJECTS=${1:-30} BF_SEQ_MODES=native timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/fseq_prof -o fseq -- python3 scripts/fusion_seq_bench.py 6
