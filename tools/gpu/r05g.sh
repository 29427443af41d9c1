set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
for sh in "65536 320 2560 39 1 0" "65536 320 2560 32 1 0" "65536 320 960 39 0 0" "65536 320 960 32 0 0" "65536 320 320 39 0 1" "65536 320 320 34 0 1" "65536 1280 320 39 0 1" "65536 1280 320 37 0 1" "16384 640 5120 39 1 0" "16384 640 5120 32 1 0" "4096 1280 10240 39 1 0" "4096 1280 10240 32 1 0" "16384 2560 640 39 0 1" "4096 5120 1280 39 0 1" "16384 640 640 39 0 1" "4096 1280 1280 39 0 1" "16384 640 1920 39 0 0" "4096 1280 3840 39 0 0"; do
  timeout -k 5 60 tools/dma_stamps $sh >> $O/dma_stamps.jsonl 2>> $O/err.txt || { echo "dma stamps failed $sh"; tail $O/err.txt; exit 5; }
done
python3 -c "
import json
for l in open('$O/dma_stamps.jsonl'):
    d=json.loads(l); c=d['cycles']
    print(d['shape'], 't',d['tile'],'geglu',d['geglu'],'res',d['res'],'us',d['us'],'TF',d['tflops'],'kloop',c['kloop_med'],'epi',c['epilogue_med'],'blk',c['block_med'])
"
timeout -k 10 900 python3 -u -m pytest tests/test_tiles_gpu.py tests/test_kernels_gpu.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 4; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 6; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r['launches_per_step'])"
