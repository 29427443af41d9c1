#!/bin/bash
# r06 validation (RDEIC_HEAD=<commit> names the tree in the profiles) in ONE call: the driver's gpu tests, smoke, the default bench line,
# a rocprofv3 kernel trace of the bench (step slice + conv cross-check), and the PMC HBM traffic passes.
# usage (repo root on the box): RDEIC_HEAD=$(git rev-parse --short HEAD) bash tools/gpu/r06_round.sh TAG
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
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 5; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('algorithmic_bytes_per_launch'))"
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof failed"; tail -20 $O/bench_prof.err; exit 7; }
cd $R
python3 tools/step_kernels.py $O/prof/bench_kernel_trace.csv --bench $O/bench_prof.json --out $O/step_kernels.json > $O/step_kernels.txt || { echo "step slice failed"; exit 8; }
python3 -c "import json;d=json.load(open('$O/step_kernels.json'));print('step', d['span_ms'], d['kernel_busy_ms'], d['families']['conv'], d.get('conv_crosscheck'))"
bash tools/pmc_bench.sh $TAG/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 9; }
tail -3 $O/pmc.log
