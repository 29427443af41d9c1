#!/bin/bash
# r04: halo8 main-loop decomposition on the 256^2 x 256 layer. diag bits removed per build:
# 59 = waits+barriers+transform+reads+DMA (MFMA only), 51 = all but the transform, 57 = all but the
# barriers, 43 = all but the LDS fragment reads; cur = the default
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
run() {  # name binary
  for cfg in "16 256 256 256 256 1 1" "16 512 512 128 128 1 1"; do
    echo -n "{\"v\": \"$1\", \"r\": " >> $O/halo.jsonl
    timeout -k 5 60 tools/halo_stamps_$2 $cfg >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps $1 failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo.jsonl
  done
}
for rep in 1 2; do
  run cur cur
  run mfma_only diag59
  run plus_transform diag51
  run plus_barriers diag57
  run plus_reads diag43
done
python - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open('gpurun_out/r04t/halo.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    agg[(d['v'], r['shape'][1], r['shape'][3])].append((r['ms'], c['main_med'], c['block_med'], c['epilogue_med']))
for k, v in agg.items():
    print(k, 'ms', round(sum(x[0] for x in v)/len(v), 4), 'main', sorted(x[1] for x in v)[0], 'block', sorted(x[2] for x in v)[0], 'epi', sorted(x[3] for x in v)[0])
PY
