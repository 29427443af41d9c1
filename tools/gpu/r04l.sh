#!/bin/bash
# r04: halo8 2-tap barriers (sp3b2) vs balanced transform (sp3); halo tests on the sp3+bar2 library build
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
for v in sp3 b2; do
  RDEIC_LIB=$PWD/rdeic_amd/lib_$v/librdeic_hip.so timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_halo_conv_gpu.py > $O/pytest_$v.log 2>&1 || { echo "halo tests ($v) failed"; tail -30 $O/pytest_$v.log; exit 4; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
run() {  # name binary env
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1" "16 64 64 512 512 1 1" "16 512 512 256 128 1 1"; do
    echo -n "{\"v\": \"$1\", \"r\": " >> $O/halo.jsonl
    env $3 timeout -k 5 60 tools/halo_stamps_$2 $cfg >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo.jsonl
  done
}
for rep in 1 2; do
  run halo4 d0 HALO4=1
  run halo8_sp3 sp3 HALO4=0
  run halo8_sp3_bar2 sp3b2 HALO4=0
done
python - <<'PY'
import json
for l in open('gpurun_out/r04l/halo.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    print(d['v'], r['shape'][1], r['shape'][3], r['shape'][4], r['ms'], r['tflops'], r['tile_rows'], c['prologue_med'], c['main_med'], c['epilogue_med'], c['block_med'], r['main_floor_cycles'])
PY
