# One GPU call: gpu tests, smoke, bench line, rocprofv3 kernel stats of the bench.
# usage (repo root on the box): bash tools/gpu_round.sh TAG [tests|notests]
set -e
TAG=${1:-run}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "${2:-tests}" = "tests" ]; then
  # exactly the driver's command (no extra flags or env)
  timeout -k 10 600 python3 -m pytest tests/ -x -q -m gpu > $O/pytest.log 2>&1
  echo "tests ok"
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
  echo "smoke ok"
fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err
echo "prof ok"
cd $R
python tools/step_kernels.py $O/prof/bench_kernel_trace.csv --bench $O/bench_prof.json --out $O/step_kernels.json > /dev/null
echo "step summary ok"
