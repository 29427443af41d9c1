#!/bin/bash
# r06: conv option A/B in the concurrent bench (driver counts), alternating on one box.
# usage: bash tools/gpu/r06ab.sh TAG "K=V" [REPS]
set -o pipefail
TAG=${1:-r06ab}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
for rep in $(seq 1 ${3:-3}); do
  for v in base opt; do
    A=""; [ $v = opt ] && A="--conv-option $2"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 $A > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v $rep', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
