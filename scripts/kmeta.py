"""Per-kernel VGPR / scratch / LDS from a hipcc device .s (amdhsa metadata)."""
import re
import sys
txt = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n  - \.", txt.split("amdhsa.kernels:")[1]):
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or pat not in name.group(1):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print(f"{name.group(1)[:60]:60s} vgpr {g('vgpr_count'):>4} scratch {g('private_segment_fixed_size'):>4} "
          f"lds {g('group_segment_fixed_size'):>6} spill {g('vgpr_spill_count')}")
