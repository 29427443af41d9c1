#!/bin/bash
# r06: tiled checkerboard entropy kernels: bitstream / entropy tests, then the bench's step slice (entropy family)
set -o pipefail
TAG=${1:-r06u}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_e2e_gpu.py tests/test_config2_gpu.py tests/test_kernels_gpu.py tests/test_cli_gpu.py tests/test_sessions_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof failed"; tail -20 $O/bench_prof.err; exit 7; }
cd $R
python3 tools/step_kernels.py $O/prof/bench_kernel_trace.csv --bench $O/bench_prof.json --out $O/step_kernels.json > $O/step_kernels.txt || { echo "step slice failed"; exit 8; }
python3 -c "import json;d=json.load(open('$O/step_kernels.json'));print('step', d['span_ms'], d['kernel_busy_ms'], d['families'])"
