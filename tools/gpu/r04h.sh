#!/bin/bash
# r04: halo conv variants on one box: 4-row (HALO4), 8-row burst transform, 8-row spread-after-MFMA, 8-row no transform
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
run() {  # name binary env
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1"; do
    echo -n "{\"v\": \"$1\", \"r\": " >> $O/halo.jsonl
    env $3 timeout -k 5 60 tools/halo_stamps_$2 $cfg >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo.jsonl
  done
}
for rep in 1 2; do
  run halo4 d0 HALO4=1
  run halo8 d0 HALO4=0
  run halo8_spread sp HALO4=0
  run halo8_notransform d8 HALO4=0
done
python - <<'PY'
import json
for l in open('gpurun_out/r04h/halo.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    print(d['v'], r['shape'][1], r['shape'][3], r['ms'], r['tflops'], r['tile_rows'], c['prologue_med'], c['main_med'], c['epilogue_med'], c['block_med'], r['main_floor_cycles'])
PY
