#!/bin/bash
# r04: halo8 main-loop bounds (diag builds: 16 no LDS fragment reads, 33 no DMA and no waits, 49 both)
# against the default build; then the UNet-ResBlock GN+SiLU fusion A/B (tools/halo_bench.py unet)
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
run() {  # name binary
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1"; do
    echo -n "{\"v\": \"$1\", \"r\": " >> $O/halo.jsonl
    timeout -k 5 60 tools/halo_stamps_$2 $cfg >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps $1 failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo.jsonl
  done
}
for rep in 1 2; do
  run default cur
  run no_lds_reads diag16
  run no_dma_no_waits diag33
  run no_dma_no_reads diag49
done
python - <<'PY'
import json
for l in open('gpurun_out/r04n/halo.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    print(d['v'], r['shape'][1], r['shape'][3], r['shape'][4], r['ms'], r['tflops'], c['prologue_med'], c['main_med'], c['epilogue_med'], c['block_med'], r['main_floor_cycles'])
PY
timeout -k 10 300 python -u tools/halo_bench.py unet > $O/unet_ab.txt 2>&1 || { echo "unet A/B failed"; tail -20 $O/unet_ab.txt; exit 4; }
grep -v amdgpu.ids $O/unet_ab.txt
