#!/bin/bash
# r06: focused tests (edge convs, fused GroupNorm, config 2), a bench A/B against ab/r05, layer times, and the
# rocprofv3 kernel trace of the bench sliced to its last single-session step.
# usage (repo root on the box): bash tools/gpu/r06c.sh TAG
set -o pipefail
TAG=${1:-r06c}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_edge_convs_gpu.py tests/test_gn_fused_gpu.py tests/test_config2_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/new1.json 2> $O/new1.err || { echo "bench new failed"; tail -20 $O/new1.err; exit 5; }
python3 -c "import json;d=json.load(open('$O/new1.json'));r=d['roofline'];print('new1', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
(cd ab/r05 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/r05_1.json 2> $O/r05_1.err) || { echo "bench r05 failed"; tail -20 $O/r05_1.err; exit 5; }
python3 -c "import json;d=json.load(open('$O/r05_1.json'));r=d['roofline'];print('r05_1', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
timeout -k 10 300 python -u tools/layer_times.py > $O/layer_times_new.txt 2> $O/lt_new.err || { echo "layer_times failed"; tail -20 $O/lt_new.err; exit 7; }
grep -E "512, 512, 8, 128|512, 512, 128, 3," $O/layer_times_new.txt
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof failed"; tail -20 $O/bench_prof.err; exit 8; }
cd $R
python3 tools/step_kernels.py $O/prof/bench_kernel_trace.csv --bench $O/bench_prof.json --out $O/step_kernels.json > $O/step_kernels.txt || { echo "step slice failed"; exit 9; }
python3 -c "import json;d=json.load(open('$O/step_kernels.json'));print('step', d['span_ms'], d['kernel_busy_ms'], {k: v for k, v in d['families'].items() if k in ('conv', 'groupnorm', 'attention', 'layernorm')})"
