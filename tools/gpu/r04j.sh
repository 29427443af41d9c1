#!/bin/bash
# r04: halo8 transform balanced over all 16 waves (sp3) vs loader-only spread (sp)
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
run() {  # name binary env
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1"; do
    echo -n "{\"v\": \"$1\", \"r\": " >> $O/halo.jsonl
    env $3 timeout -k 5 60 tools/halo_stamps_$2 $cfg >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo.jsonl
  done
}
for rep in 1 2; do
  run halo8_sp sp HALO4=0
  run halo8_sp3 sp3 HALO4=0
  run halo8_sp3_nobarrier sp3nb HALO4=0
done
python - <<'PY'
import json
for l in open('gpurun_out/r04j/halo.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    print(d['v'], r['shape'][1], r['shape'][3], r['ms'], r['tflops'], r['tile_rows'], c['prologue_med'], c['main_med'], c['epilogue_med'], c['block_med'], r['main_floor_cycles'])
PY
