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
# busy fraction per 50-ms bucket (the timed region shows as the long run of high buckets)
B = 50_000_000
nb = int(span // B) + 1
acc = [0] * nb
t_start = iv[0][0]
cs, ce = iv[0]
merged = []
for s_, e_ in iv[1:]:
    if s_ > ce:
        merged.append((cs, ce))
        cs, ce = s_, e_
    else:
        ce = max(ce, e_)
merged.append((cs, ce))
for s_, e_ in merged:
    while s_ < e_:
        k = int((s_ - t_start) // B)
        edge = t_start + (k + 1) * B
        acc[k] += min(e_, edge) - s_
        s_ = min(e_, edge)
print("busy % per 50 ms:", " ".join(f"{100 * a / B:.0f}" for a in acc))
print(f"span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms ({100 * busy / span:.1f} %), "
      f"{len(gaps)} gaps, {sum(gaps) / 1e6:.2f} ms idle; gaps > 20 us: {len(big)} totalling "
      f"{sum(big) / 1e6:.2f} ms; largest {[round(g / 1e3) for g in gaps[-8:]]} us")
