#!/bin/bash
# A/B of a runtime environment setting on the driver-form bench (interleaved, same box).
# usage (repo root on the box): bash tools/gpu/env_ab.sh TAG "VAR=VALUE" [REPS]
set -o pipefail
O=$PWD/gpurun_out/${1:-env_ab}
mkdir -p $O
for rep in $(seq 1 ${3:-2}); do
  for v in base env; do
    E=""; [ $v = env ] && E="$2"
    env $E timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 --no-roofline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v $rep', d['value'], d['ms_per_step'])"
  done
done
