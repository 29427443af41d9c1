#!/bin/bash
# r06: same-box A/B of the round-5 final tree (ab/r05tree) against HEAD, alternating, and a codec-session sweep
set -o pipefail
TAG=${1:-r06v}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
for i in 1 2 3; do
  (cd ab/r05tree && timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/r05_$i.json 2> $O/r05_$i.err) || { echo "r05 bench failed"; tail -5 $O/r05_$i.err; exit 3; }
  python3 -c "import json; d=json.loads(open('$O/r05_$i.json').read().strip().splitlines()[-1]); print('r05_$i', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/head_$i.json 2> $O/head_$i.err || { echo "head bench failed"; tail -5 $O/head_$i.err; exit 4; }
  python3 -c "import json; d=json.loads(open('$O/head_$i.json').read().strip().splitlines()[-1]); print('head_$i', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
for st in 4 6 8; do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --fp32-steps 0 --streams $st > $O/s$st.json 2> $O/s$st.err || { echo "streams $st failed"; tail -5 $O/s$st.err; exit 5; }
  python3 -c "import json; d=json.loads(open('$O/s$st.json').read().strip().splitlines()[-1]); print('streams $st', d['value'], d['ms_per_step'])"
done
