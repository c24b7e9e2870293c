#!/bin/bash
# PMC passes over any command; per-dispatch averages of the kernels whose name contains FILTER.
# usage: scripts/pmc_run.sh <tag> <filter> <python script> [args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; filt=$2; shift 2
out=gpurun_out/pmc_$tag; mkdir -p $out
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d /tmp/pmc_${tag}_$i -o p -- python3 "$@" > $out/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/pass$i.log; exit 1; }
  f=$(find /tmp/pmc_${tag}_$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$out/pass$i.txt" "$filt" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
disp = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if sys.argv[3] not in r['Kernel_Name']:
        continue
    disp[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
ids = sorted(disp, key=int)[2:] or sorted(disp, key=int)
names = sorted({n for d in disp.values() for n in d})
with open(sys.argv[2], 'w') as f:
    for n in names:
        vals = [disp[i][n] for i in ids]
        line = f"{n:32s} {sum(vals)/len(vals):.4g}"
        print(line); f.write(line + "\n")
PY
done
