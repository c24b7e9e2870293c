#!/bin/bash
# Regenerate the committed profiles of a round on the GPU box:
#   profiles/<r>_bench_kernel_stats.csv / _domain_stats.csv   rocprofv3 --kernel-trace --stats of bench.py
#   profiles/<r>_bench_under_rocprof.json                      the bench line of that same run
#   profiles/<r>_roofline_kernel_stats.csv / _roofline_bench.json  eager single-stream run: the
#                                                              bench timer's launches = the trace's
#   profiles/<r>_pmc.json       HBM-side bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, separate
#                               --pmc passes) per kernel name and for the bench line's roofline
#                               kernels; SQ instruction mix of the attention kernels
#   profiles/<r>_bench_default.json                            a plain bench run
# usage: scripts/profile_round.sh r02 [all|pmc|trace]
set -o pipefail
R=${1:-r02}
ONLY=${2:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof_$R gpurun_out/profiles
P=gpurun_out/profiles     # copied into profiles/ afterwards (only gpurun_out/ comes back from the box)

if [ "$ONLY" = all ] || [ "$ONLY" = trace ]; then
echo "== kernel trace"
rm -rf /tmp/kt_$R
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$R -o run -- \
    python3 -u bench.py --no-cpu-baseline --steps 40 > gpurun_out/prof_$R/kt.log 2>&1 || { tail -20 gpurun_out/prof_$R/kt.log; exit 1; }
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

if [ "$ONLY" = all ] || [ "$ONLY" = pmc ]; then
# PMC_EXTRA: extra bench flags for a workload's own PMC file (e.g. R=r02_fp8 PMC_EXTRA="--clip-fp8 --vocab 200")
PMC_CMD="python3 -u bench.py --steps 2 --warmup 1 --eager --inflight 1 --no-cpu-baseline --roofline-steps 1 ${PMC_EXTRA:-}"
# SQ_PASS: an extra pass of SQ counters (names as `rocprofv3 -L` lists them on the box)
for pass in FETCH_SIZE WRITE_SIZE ${SQ_PASS:+"$SQ_PASS"}; do
  tag=$(echo $pass | cut -d' ' -f1)
  echo "== pmc $pass"
  rm -rf /tmp/pmc_${R}_$tag
  timeout -s KILL 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/pmc_${R}_$tag -o p -- \
      $PMC_CMD > gpurun_out/prof_$R/pmc_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$R/pmc_$tag.log; exit 1; }
done
python3 - "$R" <<'PY'
import csv, glob, json, re, sys, collections
R = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for d in sorted(glob.glob(f"/tmp/pmc_{R}_*")):
    fs = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    f = fs[0]
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"]][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
kernels = {}
for name, ctrs in per.items():
    k = {}
    for c, d in ctrs.items():
        k[c] = sum(d.values()) / max(len(d), 1)
        k[c + "_dispatches"] = len(d)
    if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
        k["bytes_per_launch"] = (2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024
    kernels[name] = k
# the bench line's roofline kernels: launch-weighted averages over the matching kernel names
# (regular expressions over the demangled names; k_gemm256p<OUT_BF16, ACT, F8>)
# (k_gemm256q, the overlapped-epilogue form, runs the bf16-output GEMMs from round 3 on: it joins
# the bf16 GEMM groups under the same keys)
# (round 5: hand-written kernels only; k_gemm256q<OUT_BF16, ACT, RES, F8, MB1> at every tile height)
groups = {"k_gemm256p": [r"k_gemm256p<\w+, \d, 0>", r"k_gemm256q<\w+, \d, \w+, 0"],
          "k_gemm256p<false, 0>": [r"k_gemm256p<false, 0, 0>", r"k_gemm256q<false, 0, true"],
          "k_gemm256p<true, 1>": [r"k_gemm256p<true, 1, 0>", r"k_gemm256q<true, 1, false, 0"],
          "k_gemm256p_fp8": [r"k_gemm256p<\w+, \d, [13]>", r"k_gemm256q<\w+, \d, \w+, [13]"],
          "k_attn": ["k_attn"],
          "k_attn_clip": ["k_attn2<80"],
          "k_attn_cutr": ["k_attn2<64"]}
out = {"round": int(re.match(r"r(\d+)", R).group(1)), "workload": R, "method": (
    "rocprofv3 --pmc FETCH_SIZE --kernel-trace, a separate --pmc WRITE_SIZE pass and an SQ "
    "instruction-count pass over `bench.py --steps 2 --warmup 1 --eager --inflight 1`; per-dispatch "
    "values summed over the XCD instances and averaged over the dispatches of a kernel name; "
    "bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) KiB -> bytes (gfx950 tallies 128-B reads at "
    "64 B, MI355X_MICROARCH.md HBM section).  Memory-side L2 traffic, Infinity-Cache hits included."),
    "kernels": kernels}
for key, pats in groups.items():
    sel = [(n, k) for n, k in kernels.items() if any(re.search(p, n) for p in pats) and "bytes_per_launch" in k]
    if not sel:
        continue
    w = sum(k["FETCH_SIZE_dispatches"] for _, k in sel)
    out[key] = {"bytes_per_launch": sum(k["bytes_per_launch"] * k["FETCH_SIZE_dispatches"] for _, k in sel) / w,
                "dispatches": w, "kernel_names": [n for n, _ in sel]}
json.dump(out, open(f"gpurun_out/profiles/{R}_pmc.json", "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))
PY
[ $? -eq 0 ] || exit 1
fi

if [ "$ONLY" = all ]; then
echo "== bench default"
timeout -k 10 400 python3 -u bench.py > gpurun_out/prof_$R/default.log 2>&1 || { tail -20 gpurun_out/prof_$R/default.log; exit 1; }
grep '"metric"' gpurun_out/prof_$R/default.log > $P/${R}_bench_default.json
cat $P/${R}_bench_default.json
fi
