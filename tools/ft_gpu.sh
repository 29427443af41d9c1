# Fine-tune step checks on one GPU: kernel-level backward tests, then the golden-step parity test.
# usage: bash tools/ft_gpu.sh TAG   (stops after a crash / timeout; pytest failures (rc 1) continue)
set -u
O=gpurun_out/${1:-ft}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_train_kernels_gpu.py -v --timeout 200 --timeout-method thread > $O/kern.log 2>&1
rc=$?
tail -8 $O/kern.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: kernel tests rc=$rc"; exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_finetune_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -30 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: fine-tune tests rc=$rc"; exit $rc; fi
timeout -k 10 240 python -u bench_train.py --steps 3 --warmup 1 > $O/bench_train_fp32.json 2> $O/bench_train_fp32.err
rc=$?
cat $O/bench_train_fp32.json; tail -3 $O/bench_train_fp32.err
if [ $rc -ne 0 ]; then echo "stop: bench_train fp32 rc=$rc"; exit $rc; fi
timeout -k 10 240 python -u bench_train.py --steps 3 --warmup 1 --dtype bf16 > $O/bench_train_bf16.json 2> $O/bench_train_bf16.err
rc=$?
cat $O/bench_train_bf16.json; tail -3 $O/bench_train_bf16.err
exit $rc
