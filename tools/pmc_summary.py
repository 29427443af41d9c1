"""Summarise rocprofv3 --pmc counter_collection CSVs: mean counter value per kernel name."""
import collections
import csv
import sys


def load(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


for path in sys.argv[1:]:
    print("==", path)
    for k, cs in load(path).items():
        if "conv" not in k and "attn" not in k:
            continue
        short = k.split("(")[0][-90:]
        print("  ", short)
        for c, v in sorted(cs.items()):
            print(f"      {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
