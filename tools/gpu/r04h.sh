#!/bin/bash
# r04: 8-row halo conv phase split (stamps) and attribution (4 no MFMA, 8 no transform)
set -o pipefail
O=gpurun_out/r04h
mkdir -p $O
for d in 0 4 8; do
  for cfg in "16 512 512 128 128 1 1" "16 128 128 512 512 1 1"; do
    echo -n "{\"diag\": $d, \"r\": " >> $O/halo8.jsonl
    timeout -k 5 60 tools/halo_stamps_d$d $cfg >> $O/halo8.jsonl 2>> $O/halo8.err || { echo "stamps failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo8.jsonl
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r04h/halo8.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    print(d['diag'], r['shape'][1], r['shape'][3], r['ms'], r['tflops'], r['tile_rows'], c['prologue_med'], c['main_med'], c['epilogue_med'], c['block_med'], r['main_floor_cycles'])
PY
