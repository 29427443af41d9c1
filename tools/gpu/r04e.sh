#!/bin/bash
# r04: halo transform spread over taps 2..5 vs one burst at tap 2 (both -fno-slp-vectorize)
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
for rep in 1 2; do
for v in noslp spread after; do
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1"; do
    echo -n "{\"build\": \"$v\", \"r\": " >> $O/halo.jsonl
    timeout -k 5 60 tools/halo_stamps_$v $cfg >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo.jsonl
  done
done
done
python - <<'PY'
import json
for l in open('gpurun_out/r04f/halo.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    print(d['build'], r['shape'][3], r['ms'], r['tflops'], c['prologue_med'], c['main_med'], c['epilogue_med'])
PY
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_halo_conv_gpu.py > $O/pytest.log 2>&1 || { echo "halo tests failed"; tail -30 $O/pytest.log; exit 4; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u tools/halo_bench.py unet > $O/halo_bench_unet.txt 2>&1 || { echo "halo_bench unet failed"; exit 5; }
timeout -k 10 200 python -u tools/halo_bench.py > $O/halo_bench_vae.txt 2>&1 || { echo "halo_bench vae failed"; exit 5; }
cat $O/halo_bench_unet.txt $O/halo_bench_vae.txt
