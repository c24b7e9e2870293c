#!/bin/bash
# SQ / TCC counters of one attention shape (scripts/attn_one.py), one --pmc pass per group.
# usage: scripts/attn_pmc.sh B H S D variant tag
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B=$1; H=$2; S=$3; D=$4; V=$5; TAG=${6:-attn}
mkdir -p gpurun_out/pmc_$TAG
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rm -rf /tmp/apmc_$i
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/apmc_$i -o p -- \
      python3 -u scripts/attn_one.py $B $H $S $D $V 10 > gpurun_out/pmc_$TAG/pass$i.log 2>&1 || { tail -5 gpurun_out/pmc_$TAG/pass$i.log; exit 1; }
  cp "$(find /tmp/apmc_$i -name '*counter_collection.csv' | head -1)" gpurun_out/pmc_$TAG/pass$i.csv
done
python3 - gpurun_out/pmc_$TAG <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(d + "/pass*.csv")):
    for r in csv.DictReader(open(f)):
        if "attn" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, v in agg.items():
    vals = list(v.values())[2:]      # skip the first launches
    print(f"{c:28s} {sum(vals)/max(len(vals),1):16.1f}")
PY
