#!/bin/bash
# r06: three-way bench A/B, alternating on one box: A = previous lib + previous tile table, B = current lib +
# current table, C = current lib + previous table
set -o pipefail
TAG=${1:-r06t}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
for i in 1 2 3; do
  for T in A B C; do
    case $T in
      A) L=$R/ab/old/librdeic_hip.so; TT=$R/ab/old/conv_tiles_pre.json;;
      B) L=$R/rdeic_amd/lib/librdeic_hip.so; TT=$R/rdeic_amd/conv_tiles.json;;
      C) L=$R/rdeic_amd/lib/librdeic_hip.so; TT=$R/ab/old/conv_tiles_pre.json;;
    esac
    RDEIC_LIB=$L RDEIC_TILE_TABLE=$TT timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/$T$i.json 2> $O/$T$i.err || { echo "bench $T$i failed"; tail -5 $O/$T$i.err; exit 7; }
    python3 -c "import json; d=json.loads(open('$O/$T$i.json').read().strip().splitlines()[-1]); print('$T$i', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
