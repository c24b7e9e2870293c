"""Golden fixture for the result writers: runs the REFERENCE tools/utils.py post_process
(tools/utils.py:302-317) on seeded corner sets.  Only absent third-party modules imported by
tools/utils.py at module level are replaced (rerun, open3d, cv2, torchvision, none of them used by
post_process).  Run:  python tests/golden/make_golden_results.py  ->  tests/golden/results.npz
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("BOXFUSION_REFERENCE", "/root/reference")
sys.path.insert(0, HERE)
sys.path.insert(0, REF)
import make_golden  # noqa: E402,F401  (torchvision / cv2 / pycuda stand-ins)

for name in ("rerun", "rerun.blueprint", "open3d", "torchvision.transforms.functional"):
    if name not in sys.modules:
        try:
            __import__(name)
        except Exception:
            sys.modules[name] = types.ModuleType(name)
sys.modules["torchvision.transforms.functional"].pil_to_tensor = lambda *a, **k: None
sys.modules["rerun"].blueprint = sys.modules["rerun.blueprint"]

from tools import utils as U  # noqa: E402


def main():
    rng = np.random.default_rng(7)
    n = 200
    lo = rng.uniform(-3, 3, (n, 1, 3)).astype(np.float32)
    ext = rng.uniform(0.0, 0.8, (n, 1, 3)).astype(np.float32)
    ext[:10] = 0.3                                   # exactly at the threshold
    ext[10:20, :, 1] = np.float32(0.3) - np.float32(1e-7)
    corners = lo + ext * rng.uniform(0, 1, (n, 8, 3)).astype(np.float32)
    corners[:, 0] = lo[:, 0]
    corners[:, 1] = lo[:, 0] + ext[:, 0]
    out = U.post_process(corners.copy())
    out_t = U.post_process(corners.copy(), threshold=0.5)
    np.savez_compressed(os.path.join(HERE, "results.npz"), corners=corners, post=out, post_05=out_t)
    print("results.npz:", corners.shape, "->", out.shape, out_t.shape)


if __name__ == "__main__":
    main()
