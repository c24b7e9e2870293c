#!/bin/bash
# rank 0's configuration at 8 ranks (--sim-ranks 8: one GPU detecting rank 0's frames and fusing all
# 8 ranks' keyframes) against the N = 1 step on the same box: CU reservation + 7 frames (the
# round-4 default), no reservation + 8 frames, reservation + 8 frames.
mkdir -p gpurun_out/sim8ab
for w in "n1:--steps 40" "res7:--sim-ranks 8 --steps 40" "nores8:--sim-ranks 8 --steps 40 --fusion-cus 0 --rank0-batch 8" \
         "res8:--sim-ranks 8 --steps 40 --rank0-batch 8" "n1b:--steps 40"; do
  n=${w%%:*}; a=${w#*:}
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > gpurun_out/sim8ab/$n.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/sim8ab/$n.log; exit 1; }
  python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/sim8ab/{n}.log") if l.startswith("{")][-1])
print(n, round(d["ms_per_step"], 2), "ms/step", round(d["value"], 1), "frames/s; worker",
      (d.get("fusion_owner") or {}).get("busy_ms_per_step"), "ms/step; rank0_batch", d["config"].get("rank0_batch"))
PY
done
