#!/bin/bash
# Same-box A/B of halo-conv builds (tools/halo_stamps.hip compiled with different RDEIC_HALO8_* /
# RDEIC_HALO_DIAG switches, e.g. tools/halo_stamps_cur, tools/halo_stamps_diag33), interleaved over
# REPS rounds on the VAE ResnetBlock shapes; prints per-variant mean ms and median cycles.
# usage (repo root on the box): bash tools/gpu/halo_ab.sh TAG REPS name:binary[:ENV=VAL] ...
#   e.g. bash tools/gpu/halo_ab.sh r04o 3 cur:cur vf:vf tw4:tw4 halo4:cur:HALO4=1
set -o pipefail
O=gpurun_out/$1
REPS=$2
shift 2
mkdir -p $O
SHAPES=${HALO_AB_SHAPES:-"16,512,512,128,128 16,256,256,256,256 16,128,128,512,512 16,512,512,256,128"}
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS=: read -r name bin envs <<< "$spec"
    for sh in $SHAPES; do
      echo -n "{\"v\": \"$name\", \"r\": " >> $O/halo.jsonl
      env $envs timeout -k 5 60 tools/halo_stamps_$bin ${sh//,/ } 1 1 >> $O/halo.jsonl 2>> $O/halo.err || { echo "stamps $name failed"; exit 3; }
      sed -i '$ s/$/}/' $O/halo.jsonl
    done
  done
done
python3 - $O/halo.jsonl <<'PY'
import json, collections, sys
agg = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r = d['r']; c = r['cycles']
    agg[(d['v'], r['shape'][1], r['shape'][3], r['shape'][4])].append((r['ms'], c['main_med'], c['block_med'], c['epilogue_med'], c['prologue_med'], r.get('epi_overlap', 0)))
for k, v in agg.items():
    med = lambda i: sorted(x[i] for x in v)[len(v) // 2]
    print(k, 'ms', round(sum(x[0] for x in v) / len(v), 4), 'pro', med(4), 'main', med(1), 'epi', med(3), 'block', med(2), 'epi_overlap', med(5))
PY
