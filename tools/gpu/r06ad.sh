#!/bin/bash
# r06: tile of the fine-tune step's split-K partial launches (conv option 12), alternating on one box
set -o pipefail
TAG=${1:-r06ad}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  for v in base 30 36 38 37 25; do
    A=""; [ $v != base ] && A="--conv-option 12=$v"
    timeout -k 10 300 python -u bench_train.py --dtype bf16 --no-roofline $A > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "ft $v failed"; tail -5 $O/${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$rep.json')); print('$v $rep', d['value'], d['ms_per_step'], d['config']['mean_loss'])"
  done
done
