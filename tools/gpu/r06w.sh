#!/bin/bash
# r06: codec sessions in flight, alternating 5 / 8 / 12 on one box
set -o pipefail
TAG=${1:-r06w}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
for i in 1 2 3; do
  for st in ${SESS_LIST:-5 8 12}; do
    timeout -k 10 300 python -u bench.py --steps ${K:-8} --warmup ${W:-2} --no-cpu-baseline --fp32-steps 0 --streams $st > $O/s${st}_$i.json 2> $O/s${st}_$i.err || { echo "streams $st failed"; tail -5 $O/s${st}_$i.err; exit 5; }
    python3 -c "import json; d=json.loads(open('$O/s${st}_$i.json').read().strip().splitlines()[-1]); print('streams $st', d['value'], d['ms_per_step'])"
  done
done
