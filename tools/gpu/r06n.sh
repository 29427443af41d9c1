#!/bin/bash
# r06: config-5 split-K policy A/B (alternating, same box)
set -o pipefail
TAG=${1:-r06n}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  for pol in short long off; do
    timeout -k 10 300 python -u bench_train.py --dtype bf16 --ft-splitk $pol --no-roofline > $O/ft_$pol.$rep.json 2> $O/ft_$pol.$rep.err || { echo "ft $pol failed"; tail -20 $O/ft_$pol.$rep.err; exit 3; }
    python3 -c "import json;d=json.load(open('$O/ft_$pol.$rep.json'));print('$pol', d['value'], d['ms_per_step'], d['config']['mean_loss'])"
  done
done
