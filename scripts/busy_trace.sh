#!/bin/bash
# kernel trace of a default bench run and the GPU busy fraction over its timed part
# usage: scripts/busy_trace.sh [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf /tmp/kt_busy
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt_busy -o run -- \
    python3 -u bench.py --no-cpu-baseline "$@" > gpurun_out/busy_bench.log 2>&1 || { tail -5 gpurun_out/busy_bench.log; exit 1; }
f=$(find /tmp/kt_busy -name '*kernel_trace.csv' | head -n 1)
[ -n "$f" ] || { echo "no kernel trace"; exit 1; }
python3 scripts/busy_union.py "$f" 0.3
