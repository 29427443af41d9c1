"""GPU busy vs idle from a rocprofv3 kernel-trace CSV: sums kernel time and the gaps between
consecutive kernels (per stream-agnostic timeline), for a timeline slice."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ev = ev[skip:]
busy = sum(e - s for s, e, _ in ev)
span = ev[-1][1] - ev[0][0]
gaps = [ev[i + 1][0] - ev[i][1] for i in range(len(ev) - 1)]
big = sorted(((g, ev[i][2][:60], ev[i + 1][2][:60]) for i, g in enumerate(gaps)), reverse=True)[:12]
print(f"kernels {len(ev)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {(span - busy) / 1e6:.2f} ms")
print(f"gaps: >50us {sum(g for g in gaps if g > 50000) / 1e6:.2f} ms, <=50us {sum(g for g in gaps if 0 < g <= 50000) / 1e6:.2f} ms")
for g, a, b in big:
    print(f"  {g / 1e3:9.1f} us after {a} -> {b}")
