#!/bin/bash
# r06: fine-tune changes: the fine-tune / training-kernel / DDP tests, then the config-5 bench and its launch census
set -o pipefail
TAG=${1:-r06y}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_finetune_gpu.py tests/test_train_kernels_gpu.py tests/test_train_cli_gpu.py tests/test_parallel_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
for i in 1 2; do
  timeout -k 10 300 python -u bench_train.py --dtype bf16 > $O/ft_$i.json 2> $O/ft_$i.err || { echo "ft failed"; tail -20 $O/ft_$i.err; exit 5; }
  python3 -c "import json;d=json.load(open('$O/ft_$i.json'));print('config5', d['value'], d['ms_per_step'], d['config']['mean_loss'])"
done
bash tools/gpu/r06l.sh $TAG/train > $O/train_trace.log 2>&1 || { echo "train trace failed"; tail -20 $O/train_trace.log; exit 6; }
head -2 $O/train_trace.log
