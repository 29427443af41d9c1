# A/B of bench variants in one GPU call (no CPU baseline; pass --no-roofline to drop the events).
# usage: bash tools/ab_bench.sh TAG "--coder-groups 1" "--coder-groups 2" ...
set -e
TAG=$1; shift
O=$PWD/gpurun_out/$TAG
mkdir -p $O
i=0
for v in "$@"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --warmup 2 $v > $O/ab$i.json 2> $O/ab$i.err
  python -c "import json,sys; d=json.load(open('$O/ab$i.json')); print('$v'.ljust(40), d['value'], d['ms_per_step'])"
  i=$((i+1))
done
