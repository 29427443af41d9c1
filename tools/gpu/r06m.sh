#!/bin/bash
# r06: config-3 bench line (1024^2, batch 8, 5 DDIM steps) and the config-5 fine-tune bench + its launch kinds
set -o pipefail
TAG=${1:-r06m}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u bench.py --size 1024 --batch 8 --ddim-steps 5 --steps 3 --warmup 1 --fp32-steps 0 --no-cpu-baseline > $O/bench_config3.json 2> $O/bench_config3.err || { echo "config3 bench failed"; tail -20 $O/bench_config3.err; exit 5; }
python3 -c "import json;d=json.load(open('$O/bench_config3.json'));print('config3', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 400 python -u bench_train.py --dtype bf16 > $O/bench_train_bf16.json 2> $O/bench_train_bf16.err || { echo "train bench failed"; tail -20 $O/bench_train_bf16.err; exit 6; }
head -c 800 $O/bench_train_bf16.json; echo
bash tools/gpu/r06l.sh $TAG/l
