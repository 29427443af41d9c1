set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_gn_fused_gpu.py tests/test_train_kernels_gpu.py tests/test_finetune_gpu.py tests/test_config2_gpu.py tests/test_parallel_gpu.py tests/test_sessions_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1; grep "worst gradient error" $O/pytest.log
timeout -k 10 300 python3 -u bench_train.py --dtype bf16 --steps 20 --warmup 3 > $O/train_bf16.json 2> $O/train_bf16.err || { echo "train bench failed"; tail -5 $O/train_bf16.err; exit 5; }
python3 -c "import json;d=json.load(open('$O/train_bf16.json'));print('train', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'], d['roofline']['families'])"
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 6; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r['launches_per_step'])"
