"""Build an A/B variant of libboxfusion_hip.so: the named sources recompiled with extra -D flags,
linked with the product objects of the other sources.

usage: python scripts/build_var.py NAME "-DFOO=1 -DBAR=2" bf_gemm.hip [bf_attn.hip ...]
   -> boxfusion_amd/_build/var_NAME/libboxfusion_hip.so   (load with BF_LIB_PATH=... or ctypes)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from boxfusion_amd import build as B  # noqa: E402


def main():
    name, flags, srcs = sys.argv[1], sys.argv[2].split(), sys.argv[3:]
    B.build()
    out = os.path.join(B.BUILD, f"var_{name}")
    os.makedirs(out, exist_ok=True)
    objs = []
    for s in sorted(os.listdir(B.CSRC)):
        if not s.endswith(".hip"):
            continue
        if s in srcs:
            o = os.path.join(out, s.replace(".hip", ".o"))
            cmd = [B.hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-fPIC", "-std=c++17", "-c",
                   os.path.join(B.CSRC, s), "-o", o, "-Wno-unused-result"] + B.SOURCES.get(s, []) + flags
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode:
                sys.exit(r.stderr)
            objs.append(o)
        else:
            objs.append(os.path.join(B.BUILD, s.replace(".hip", ".o")))
    lib = os.path.join(out, "libboxfusion_hip.so")
    r = subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib] + objs,
                       capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr)
    print(lib)


if __name__ == "__main__":
    main()
