"""Busy / idle split and the largest idle gaps of the last bench step in a rocprofv3 kernel trace."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
idx = [i for i, e in enumerate(ev) if "image_mse" in e[2]]
a, b = idx[-2] + 1, idx[-1] + 1
step = ev[a:b]
span = step[-1][1] - step[0][0]
busy = sum(e - s for s, e, _ in step)
print(f"last step: span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {(span - busy) / 1e6:.2f} ms  kernels {len(step)}")
agg = {}
for s, e, n in step:
    k = re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))[:64]
    v = agg.setdefault(k, [0, 0])
    v[0] += 1
    v[1] += e - s
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    print(f"{t / 1e6:8.2f} ms {c:5d}  {k}")
gaps = sorted(((step[i + 1][0] - step[i][1], i) for i in range(len(step) - 1)), reverse=True)
for g, i in gaps[:8]:
    print(f"  gap {g / 1e3:8.1f} us at t={(step[i][1] - step[0][0]) / 1e6:6.1f} ms after {step[i][2][:60]}")
