#!/bin/bash
# r04: halo8 in-loop transform in half pieces spread to the last tap (halves_tw4 / halves_tw2) vs the default (cur) and TW 2 alone
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
run() {  # name binary
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1" "16 128 128 512 512 1 1" "16 512 512 256 128 1 1"; do
    echo -n "{\"v\": \"$1\", \"r\": " >> $O/halo.jsonl
    timeout -k 5 60 tools/halo_stamps_$2 $cfg >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps $1 failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo.jsonl
  done
}
for rep in 1 2; do
  run cur cur
  run halves_tw4 hv4
  run halves_tw2 hv2
  run tw2 tw2
done
python - <<'PY'
import json, collections
agg = collections.defaultdict(list)
for l in open('gpurun_out/r04u/halo.jsonl'):
    d=json.loads(l); r=d['r']; c=r['cycles']
    agg[(d['v'], r['shape'][1], r['shape'][3], r['shape'][4])].append((r['ms'], c['main_med'], c['block_med']))
for k, v in agg.items():
    print(k, 'ms', round(sum(x[0] for x in v)/len(v), 4), 'main', sorted(x[1] for x in v)[len(v)//2], 'block', sorted(x[2] for x in v)[len(v)//2])
PY
