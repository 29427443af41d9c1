set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_tiles_gpu.py tests/test_gn_fused_gpu.py tests/test_halo_conv_gpu.py tests/test_config2_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 4; }
tail -1 $O/pytest.log
for sh in "65536 320 2560 32 1 0" "65536 320 2560 34 1 0" "65536 320 960 32 0 0" "65536 320 320 34 0 1" "65536 1280 320 37 0 1" "16384 640 5120 32 1 0" "4096 1280 10240 32 1 0"; do
  timeout -k 5 60 tools/dma_stamps $sh >> $O/dma_stamps.jsonl 2>> $O/err.txt || { echo "dma stamps failed"; tail $O/err.txt; exit 5; }
done
python3 -c "
import json
for l in open('$O/dma_stamps.jsonl'):
    d=json.loads(l); c=d['cycles']
    print(d['shape'], 't',d['tile'],'geglu',d['geglu'],'res',d['res'],'us',d['us'],'TF',d['tflops'],'kloop',c['kloop_med'],'epi',c['epilogue_med'],'blk',c['block_med'])
"
timeout -k 10 400 python3 -u tools/grad_dump.py $O > $O/grad_dump.log 2>&1 || { echo "grad dump failed"; tail $O/grad_dump.log; exit 6; }
tail -2 $O/grad_dump.log
timeout -k 10 300 python3 -u tools/layer_times.py > $O/layer_times.txt 2>&1 || { echo "layer times failed"; exit 7; }
head -30 $O/layer_times.txt
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 8; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
