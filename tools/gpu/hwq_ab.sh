#!/bin/bash
# A/B: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) x codec sessions (--streams).
# More sessions than hardware queues share queues, so their kernels serialise.
# usage (repo root on the box): bash tools/gpu/hwq_ab.sh TAG
set -o pipefail
O=$PWD/gpurun_out/${1:-hwq_ab}
mkdir -p $O
for rep in 1 2; do
  for cfg in "4 4" "4 8" "8 4" "8 6" "8 8"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --streams $2 --no-cpu-baseline --fp32-steps 0 --no-roofline > $O/q$1_s$2_$rep.json 2> $O/q$1_s$2_$rep.err || { echo "bench q$1 s$2 failed"; tail -5 $O/q$1_s$2_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/q$1_s$2_$rep.json').read().strip().splitlines()[-1]); print('hwq $1 sessions $2 rep $rep', d['value'], d['ms_per_step'])"
  done
done
