#!/bin/bash
# r06 end-of-round validation in ONE call (RDEIC_HEAD=<commit> names the tree): the driver's gpu tests, smoke, the
# default bench line, a rocprofv3 kernel trace of the bench (step slice), the PMC HBM traffic passes, then config 3
# (1024^2, batch 8, 5 DDIM steps) and config 5 (bf16 fine-tune step) bench lines, each with its kernel trace.
# usage (repo root on the box): RDEIC_HEAD=$(git rev-parse --short HEAD) bash tools/gpu/r06_final.sh TAG
set -o pipefail
TAG=${1:-r06_final}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 6; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 5; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('single_session_ms_per_step'))"
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof failed"; tail -20 $O/bench_prof.err; exit 7; }
cd $R
python3 tools/step_kernels.py $O/prof/bench_kernel_trace.csv --bench $O/bench_prof.json --out $O/step_kernels.json > $O/step_kernels.txt || { echo "step slice failed"; exit 8; }
python3 -c "import json;d=json.load(open('$O/step_kernels.json'));print('step', d['span_ms'], d['kernel_busy_ms'], d['families']['conv'], d.get('conv_crosscheck'))"
bash tools/pmc_bench.sh $TAG/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 9; }
tail -3 $O/pmc.log
timeout -k 10 500 python -u bench.py --size 1024 --batch 8 --ddim-steps 5 --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/bench_config3.json 2> $O/bench_config3.err || { echo "config3 bench failed"; tail -20 $O/bench_config3.err; exit 10; }
python3 -c "import json;d=json.load(open('$O/bench_config3.json'));print('config3', d['value'], d['ms_per_step'], d['roofline']['frac'])"
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3 -o bench -- python3 $R/bench.py --size 1024 --batch 8 --ddim-steps 5 --steps 1 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/bench3_prof.json 2> $O/bench3_prof.err || { echo "config3 rocprof failed"; tail -20 $O/bench3_prof.err; exit 11; }
cd $R
python3 tools/step_kernels.py $O/prof3/bench_kernel_trace.csv --bench $O/bench3_prof.json --out $O/step_kernels_config3.json > $O/step_kernels_config3.txt || { echo "config3 step slice failed"; exit 12; }
python3 -c "import json;d=json.load(open('$O/step_kernels_config3.json'));print('config3 step', d['span_ms'], d['kernel_busy_ms'], d['families']['conv'])"
timeout -k 10 400 python -u bench_train.py --dtype bf16 > $O/bench_train_bf16.json 2> $O/bench_train_bf16.err || { echo "train bench failed"; tail -20 $O/bench_train_bf16.err; exit 13; }
python3 -c "import json;d=json.load(open('$O/bench_train_bf16.json'));print('config5', d['value'], d['ms_per_step'], d['roofline']['frac'])"
bash tools/gpu/r06l.sh $TAG/train > $O/train_trace.log 2>&1 || { echo "train trace failed"; tail -20 $O/train_trace.log; exit 14; }
head -3 $O/train_trace.log
