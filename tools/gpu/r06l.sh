#!/bin/bash
# r06: the config-5 fine-tune step under a kernel trace: launches per kind for one step
set -o pipefail
TAG=${1:-r06l}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o train -- python3 $R/bench_train.py --dtype bf16 --steps 3 --warmup 2 > $O/train_prof.json 2> $O/train_prof.err || { echo "train rocprof failed"; tail -20 $O/train_prof.err; exit 8; }
cd $R
python3 - "$O" <<'PY'
import csv, glob, sys
o = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(o + "/tprof/**/train_kernel_stats.csv", recursive=True)[0])))
tot = sum(int(r["Calls"]) for r in rows)
print("total launches (5 steps + setup):", tot)
rows.sort(key=lambda r: -int(r["Calls"]))
with open(o + "/train_launch_kinds.txt", "w") as f:
    for r in rows[:80]:
        f.write(f'{int(r["Calls"]):7d} {float(r["TotalDurationNs"])/1e6:9.2f} ms  {r["Name"][:120]}\n')
print(open(o + "/train_launch_kinds.txt").read()[:4000])
PY
cat $O/train_prof.json | head -c 1500
