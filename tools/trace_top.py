"""Top kernels of one training step in a rocprofv3 kernel trace (the span between the last two
launches of the step-closing kernel, default AdamW)."""
import collections
import csv
import re
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "adamw"
rows = list(csv.DictReader(open(path)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
idx = [i for i, e in enumerate(ev) if marker in e[2]]
a, b = idx[-2] + 1, idx[-1] + 1
step = ev[a:b]
span = step[-1][1] - step[0][0]
busy = sum(e - s for s, e, _ in step)
print(f"kernels {len(step)} span {span / 1e6:.2f} ms busy {busy / 1e6:.2f} ms")


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    m = re.match(r"([A-Za-z_:0-9]+(<[^()]*>)?)", n)
    return (m.group(1) if m else n)[:90]


agg = collections.defaultdict(lambda: [0, 0])
for s, e, n in step:
    k = short(n)
    agg[k][0] += 1
    agg[k][1] += e - s
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{t / 1e6:8.2f} ms  x{c:4d}  {t / c / 1e3:8.1f} us  {k}")
