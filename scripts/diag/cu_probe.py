"""Where do the workgroups of a CU-masked stream run?  (diagnostic; scripts/diag/build_cu_probe.sh)
Prints, per stream, the set of (XCC, SE, SH, CU) the probe's workgroups ran on."""
import ctypes
import os
import sys
from collections import Counter

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from boxfusion_amd import _lib  # noqa: E402

probe = ctypes.CDLL(os.path.join(os.path.dirname(_lib.__file__), "_build", "cu_probe.so"))
det, fus = _lib.partition_cus(32)
streams = {"default": torch.cuda.current_stream(), "fusion(32)": _lib.cu_masked_stream(fus),
           "detect(224)": _lib.cu_masked_stream(det),
           "every8th": _lib.cu_masked_stream(list(range(0, 256, 8))),
           "not-every8th": _lib.cu_masked_stream([c for c in range(256) if c % 8])}
for name, s in streams.items():
    out = torch.zeros(2 * 4096, dtype=torch.int32, device="cuda")
    rc = probe.cu_probe(ctypes.c_void_p(out.data_ptr()), 4096, 20000, ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc
    torch.cuda.synchronize()
    v = out.view(-1, 2).cpu().numpy()
    hw, xcc = v[:, 0], v[:, 1] & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    units = Counter(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
    per_xcc = Counter(xcc.tolist())
    print(f"{name:12s}: {len(units)} distinct CUs; workgroups per XCC {dict(sorted(per_xcc.items()))}")
    print(f"{'':12s}  CUs per XCC {dict(sorted(Counter(k[0] for k in units).items()))}")
