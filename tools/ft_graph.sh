# Graph-captured fine-tune step: parity test, then the config-5 bench (graph and eager), one GPU.
set -u
O=gpurun_out/${1:-ftg}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_finetune_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -12 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: tests rc=$rc"; exit $rc; fi
for dt in fp32 bf16; do
  timeout -k 10 240 python -u bench_train.py --steps 5 --warmup 2 --dtype $dt > $O/bench_train_$dt.json 2> $O/bench_train_$dt.err
  rc=$?
  cat $O/bench_train_$dt.json; tail -2 $O/bench_train_$dt.err
  if [ $rc -ne 0 ]; then echo "stop: bench_train $dt rc=$rc"; exit $rc; fi
done
