set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_train_kernels_gpu.py tests/test_finetune_gpu.py tests/test_halo_conv_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python3 -u bench_train.py --dtype bf16 --steps 20 --warmup 3 > $O/train_bf16.json 2> $O/train_bf16.err || { echo "train bench failed"; tail -20 $O/train_bf16.err; exit 5; }
cat $O/train_bf16.json | head -c 1500; echo
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 6; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('traffic_over_algorithmic'))"
