#!/bin/bash
# per-kernel rocprofv3 stats of scripts/depth_std_bench.py, one shape per run
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dsprof
for shp in "$@"; do
  rm -rf /tmp/dsp_$shp
  BF_DS_SHAPE=$shp timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/dsp_$shp -o run -- \
      python3 scripts/depth_std_bench.py > gpurun_out/dsprof/log_$shp 2>&1 || exit $?
  f=$(find /tmp/dsp_$shp -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/dsprof/stats_$shp.csv
  echo "== $shp"; grep -E "k_ds_" "$f" | cut -d, -f1,2,4,6,7 | sed 's/(.*)"/"/'
done
