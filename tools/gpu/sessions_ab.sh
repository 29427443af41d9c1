#!/bin/bash
# A/B of codec sessions in flight per GPU (--streams) at the driver's step counts (--steps 20 --warmup 5)
# usage (repo root on the box): bash tools/gpu/sessions_ab.sh TAG "4 5 8 10" [REPS]
set -o pipefail
O=$PWD/gpurun_out/${1:-sessions_ab}
mkdir -p $O
for rep in $(seq 1 ${3:-2}); do
  for n in $2; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --streams $n --no-cpu-baseline --fp32-steps 0 --no-roofline > $O/s${n}_$rep.json 2> $O/s${n}_$rep.err || { echo "bench s$n failed"; tail -5 $O/s${n}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/s${n}_$rep.json').read().strip().splitlines()[-1]); print('sessions $n rep $rep', d['value'], d['ms_per_step'])"
  done
done
