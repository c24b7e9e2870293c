"""Build libboxfusion_hip.so in-tree for gfx950 (hipcc, no JIT cache, no torch extension).

Per-file flags: the fusion-side kernels are compiled with -ffp-contract=off and IEEE f32
division/sqrt so every f32 expression rounds like the reference's CPU arithmetic; the MFMA
kernels keep contraction on.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libboxfusion_hip.so")
ARCH = os.environ.get("BF_OFFLOAD_ARCH", "gfx950")

EXACT = ["-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt"]
SOURCES = {
    "bf_misc.hip": [],
    "bf_geom.hip": EXACT,
    "bf_depth.hip": EXACT,
    "bf_iou3d.hip": EXACT,
    "bf_assoc.hip": EXACT,
    "bf_fusion.hip": EXACT,
    "bf_dec_native.hip": EXACT,
    "bf_ingest.hip": EXACT,
    "bf_png.hip": EXACT,
    "bf_jpeg.hip": EXACT,
    "bf_fseq.hip": EXACT,
}
EXTRA = [s for s in sorted(os.listdir(CSRC)) if s.endswith(".hip") and s not in SOURCES]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


def _compile(src, flags):
    obj = os.path.join(BUILD, src.replace(".hip", ".o"))
    path = os.path.join(CSRC, src)
    deps = [path, os.path.join(CSRC, "bf_common.h"), os.path.join(CSRC, "bf_cv2.h"),
            os.path.join(HERE, "..", "include", "boxfusion_hip.h")]
    if os.path.exists(obj) and all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in deps
                                   if os.path.exists(d)):
        return obj
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-c", path, "-o", obj,
           "-Wno-unused-result"] + flags
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose=False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    jobs = dict(SOURCES)
    for s in EXTRA:
        jobs[s] = []
    with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
        objs = list(ex.map(lambda kv: _compile(*kv), jobs.items()))
    if not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
