"""Where do the workgroups of a CU-masked stream run?  (diagnostic; bf_cu_probe in the library)
Prints, per stream, how many CUs of each XCC the probe's workgroups ran on."""
import os
import sys
from collections import Counter

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from boxfusion_amd import _lib  # noqa: E402

n = torch.cuda.get_device_properties(0).multi_processor_count
det, fus = _lib.partition_cus(32)
streams = {"default": torch.cuda.current_stream(), "fusion(32)": _lib.cu_masked_stream(fus),
           "detect(224)": _lib.cu_masked_stream(det),
           "every8th": _lib.cu_masked_stream(list(range(0, n, 8))),
           "not-every8th": _lib.cu_masked_stream([c for c in range(n) if c % 8])}
for name, s in streams.items():
    units = _lib.cu_placement(s)
    print(f"{name:12s}: {len(units)} distinct CUs; CUs per XCC {dict(sorted(Counter(k[0] for k in units).items()))}")
