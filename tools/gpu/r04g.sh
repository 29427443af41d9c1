#!/bin/bash
# r04: 8-row halo conv (one 1024-thread block per CU) vs the 4-row kernel; tests; bench
set -o pipefail
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_halo_conv_gpu.py > $O/pytest.log 2>&1 || { echo "halo tests failed"; tail -40 $O/pytest.log; exit 4; }
tail -2 $O/pytest.log
for v in after h8; do
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1" "16 64 64 512 512 1 1" "16 512 512 256 128 1 1"; do
    echo -n "{\"build\": \"$v\", \"r\": " >> $O/halo.jsonl
    timeout -k 5 60 tools/halo_stamps_$v $cfg >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo.jsonl
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r04g/halo.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    print(d['build'], r['shape'][1], r['shape'][3], r['shape'][4], r['ms'], r['tflops'])
PY
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 5; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
