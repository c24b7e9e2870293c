#!/bin/bash
# rocprofv3 kernel-trace stats of a bench run; only the summaries come back (the trace is large).
# usage: scripts/prof_bench.sh <tag> [bench args...]
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof_$tag
rm -rf /tmp/prof_$tag
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$tag -o run -- \
    python3 -u bench.py "$@" > gpurun_out/prof_$tag/bench.log 2>&1
rc=$?
for f in $(find /tmp/prof_$tag -name "*stats*.csv"); do cp "$f" gpurun_out/prof_$tag/; done
grep '"metric"' gpurun_out/prof_$tag/bench.log
ls gpurun_out/prof_$tag
exit $rc
