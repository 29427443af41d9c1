set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_halo_conv_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 4; }
tail -1 $O/pytest.log
for sh in "16 512 512 128 128 1 1" "16 512 512 128 128 0 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1"; do
  timeout -k 5 60 tools/halo_stamps_cur $sh >> $O/stamps.jsonl 2>> $O/err.txt || { echo "stamps failed"; tail $O/err.txt; exit 3; }
done
python3 -c "
import json
for l in open('$O/stamps.jsonl'):
    d=json.loads(l); c=d['cycles']
    print(d['shape'], 'res',d['res'], 'ms',d['ms'],'TF',d['tflops'],'pro',c['prologue_med'],'main',c['main_med'],'epi',c['epilogue_med'],'blk',c['block_med'])
"
for sh in "65536 320 2560 32 1 0" "65536 320 2560 34 1 0" "65536 320 960 32 0 0" "65536 320 320 34 0 1" "65536 1280 320 37 0 1" "16384 640 5120 32 1 0" "4096 1280 10240 32 1 0" "65536 320 2560 32 0 0"; do
  timeout -k 5 60 tools/dma_stamps $sh >> $O/dma_stamps.jsonl 2>> $O/err.txt || { echo "dma stamps failed"; tail $O/err.txt; exit 5; }
done
cat $O/dma_stamps.jsonl
timeout -k 10 400 python3 -u tools/grad_dump.py $O > $O/grad_dump.log 2>&1 || { echo "grad dump failed"; tail $O/grad_dump.log; exit 6; }
tail -2 $O/grad_dump.log
