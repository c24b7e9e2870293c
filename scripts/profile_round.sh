#!/bin/bash
# Regenerate the committed profiles of a round on the GPU box:
#   profiles/<r>_bench_kernel_stats.csv / _domain_stats.csv   rocprofv3 --kernel-trace --stats of bench.py
#   profiles/<r>_bench_under_rocprof.json                      the bench line of that same run
#   profiles/<r>_pmc_gelu_gemm.json                            HBM bytes per launch of the roofline kernel
#                                                              (FETCH_SIZE x2 + WRITE_SIZE, separate passes)
#   profiles/<r>_roofline_kernel_stats.csv / _roofline_bench.json  eager single-stream run: the
#                                                              bench timer's launches = the trace's
#   profiles/<r>_bench_default.json / _breakdown.json          plain bench runs
# usage: scripts/profile_round.sh r01
set -o pipefail
R=${1:-r01}
ONLY=${2:-all}      # all | pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof_$R gpurun_out/profiles
P=gpurun_out/profiles     # copied into profiles/ afterwards (only gpurun_out/ comes back from the box)
KERNEL='k_gemm256p<true, 1>'

if [ "$ONLY" = all ]; then
echo "== kernel trace"
rm -rf /tmp/kt_$R
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$R -o run -- \
    python3 -u bench.py --no-cpu-baseline > gpurun_out/prof_$R/kt.log 2>&1 || { tail -20 gpurun_out/prof_$R/kt.log; exit 1; }
cp "$(find /tmp/kt_$R -name '*kernel_stats.csv' | head -1)" $P/${R}_bench_kernel_stats.csv
cp "$(find /tmp/kt_$R -name '*domain_stats.csv' | head -1)" $P/${R}_bench_domain_stats.csv
grep '"metric"' gpurun_out/prof_$R/kt.log > $P/${R}_bench_under_rocprof.json
echo "== roofline kernel trace (eager, one detect stream: every launch the bench's HIP-event timer sees)"
rm -rf /tmp/rk_$R
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rk_$R -o run -- \
    python3 -u bench.py --eager --inflight 1 --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$R/rk.log 2>&1 || { tail -20 gpurun_out/prof_$R/rk.log; exit 1; }
cp "$(find /tmp/rk_$R -name '*kernel_stats.csv' | head -1)" $P/${R}_roofline_kernel_stats.csv
grep '"metric"' gpurun_out/prof_$R/rk.log > $P/${R}_roofline_bench.json
fi

for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $ctr"
  rm -rf /tmp/pmc_${R}_$ctr
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d /tmp/pmc_${R}_$ctr -o p -- \
      python3 -u bench.py --steps 2 --warmup 1 --eager --no-cpu-baseline --roofline-steps 1 \
      > gpurun_out/prof_$R/pmc_$ctr.log 2>&1 || { tail -20 gpurun_out/prof_$R/pmc_$ctr.log; exit 1; }
done
python3 - "$R" "$KERNEL" <<'PY'
import csv, glob, json, sys, collections
R, kern = sys.argv[1], sys.argv[2]
res = {"kernel": kern, "round": int(R[1:]),
       "method": ("rocprofv3 --pmc FETCH_SIZE --kernel-trace and a separate --pmc WRITE_SIZE pass over "
                  "`bench.py --steps 2 --warmup 1 --eager`; per-dispatch values summed over the XCD "
                  "instances, averaged over every dispatch of the kernel; FETCH_SIZE doubled (gfx950: "
                  "128-B requests tallied at 64 B, MI355X_MICROARCH.md HBM section); KiB -> bytes. "
                  "Memory-side L2 traffic, Infinity-Cache hits included.")}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"/tmp/pmc_{R}_{ctr}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    vals = list(per.values())
    res[ctr.lower() + "_kib_avg"] = sum(vals) / max(len(vals), 1)
    res[ctr.lower() + "_dispatches"] = len(vals)
res["bytes_per_launch"] = (2 * res["fetch_size_kib_avg"] + res["write_size_kib_avg"]) * 1024
json.dump(res, open(f"gpurun_out/profiles/{R}_pmc_gelu_gemm.json", "w"), indent=1)
print(json.dumps(res))
PY
[ $? -eq 0 ] || exit 1
[ "$ONLY" = all ] || exit 0

echo "== bench default"
timeout -k 10 400 python3 -u bench.py > gpurun_out/prof_$R/default.log 2>&1 || { tail -20 gpurun_out/prof_$R/default.log; exit 1; }
grep '"metric"' gpurun_out/prof_$R/default.log > $P/${R}_bench_default.json
echo "== bench breakdown"
timeout -k 10 300 python3 -u bench.py --breakdown --steps 20 --no-cpu-baseline > gpurun_out/prof_$R/brk.log 2>&1 || { tail -20 gpurun_out/prof_$R/brk.log; exit 1; }
grep '"metric"' gpurun_out/prof_$R/brk.log > $P/${R}_bench_breakdown.json
cat $P/${R}_bench_default.json
