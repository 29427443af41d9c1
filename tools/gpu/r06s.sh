#!/bin/bash
# r06: tile-table A/B (old table vs new), bench alternating on one box; then the tile tests
set -o pipefail
TAG=${1:-r06s}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
for i in 1 2 3; do
  for T in old new; do
    if [ $T = old ]; then TT=$PWD/ab/old/conv_tiles.json; else TT=$PWD/rdeic_amd/conv_tiles.json; fi
    RDEIC_TILE_TABLE=$TT timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/$T$i.json 2> $O/$T$i.err || { echo "bench $T$i failed"; tail -5 $O/$T$i.err; exit 7; }
    python3 -c "import json; d=json.loads(open('$O/$T$i.json').read().strip().splitlines()[-1]); print('$T$i', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
timeout -k 10 400 python3 -u -m pytest tests/test_tiles_gpu.py tests/test_config2_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
