# Fine-tune step: GPU tests, a kernel trace of the bf16 step, and the config-5 bench in fp32 / bf16.
# usage: bash tools/ft_perf.sh TAG
set -u
R=$PWD
O=$R/gpurun_out/${1:-ftp}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_train_kernels_gpu.py tests/test_finetune_gpu.py -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
if [ $rc -gt 1 ]; then echo "stop: tests rc=$rc"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o train -- python3 $R/bench_train.py --steps 2 --warmup 1 --dtype ${TRACE_DTYPE:-bf16} --no-roofline > $O/bt.json 2> $O/bt.err
rc=$?
echo "rocprof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
cd $R
for dt in fp32 bf16; do
  timeout -k 10 240 python -u bench_train.py --steps 5 --warmup 2 --dtype $dt > $O/bench_train_$dt.json 2> $O/bench_train_$dt.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_train_$dt.json')); print('$dt', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
done
