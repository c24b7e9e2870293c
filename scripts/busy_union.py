"""GPU busy fraction of a rocprofv3 kernel trace: union of kernel [start, end) intervals over the
span from the first to the last kernel, plus the idle gaps' size histogram.
usage: busy_union.py <kernel_trace.csv> [skip_fraction]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2      # drop the warm-up part of the run
t0 = iv[0][0] + skip * (iv[-1][1] - iv[0][0])
iv = [(max(s, t0), e) for s, e in iv if e > t0]
busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
for s, e in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
gaps.sort()
big = [g for g in gaps if g > 20000]
print(f"span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f} %), "
      f"{len(gaps)} gaps, {sum(gaps) / 1e6:.2f} ms idle; gaps > 20 us: {len(big)} totalling "
      f"{sum(big) / 1e6:.2f} ms; largest {[round(g / 1e3) for g in gaps[-8:]]} us")
