#!/bin/bash
# r06: GEGLU chunk-pair epilogue: kernel tests, linear-tile bench old vs new, bench A/B (old / new alternating)
set -o pipefail
TAG=${1:-r06p}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_tiles_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
RDEIC_LIB=$PWD/ab/old/librdeic_hip.so timeout -k 10 300 python3 -u tools/lin_bench.py geglu --ln > $O/lin_old.jsonl 2> $O/lin_old.err || { echo "lin old failed"; tail $O/lin_old.err; exit 5; }
timeout -k 10 300 python3 -u tools/lin_bench.py geglu --ln > $O/lin_new.jsonl 2> $O/lin_new.err || { echo "lin new failed"; tail $O/lin_new.err; exit 6; }
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
old = [json.loads(l) for l in open(o + "/lin_old.jsonl")]
new = [json.loads(l) for l in open(o + "/lin_new.jsonl")]
for a, b in zip(old, new):
    print(a["name"], {k: (a[k][0] if isinstance(a[k], list) else a[k], b[k][0] if isinstance(b[k], list) else b[k]) for k in a if k != "name"})
PY
for i in 1 2 3; do
  for T in old new; do
    if [ $T = old ]; then L=$PWD/ab/old/librdeic_hip.so; TT=$PWD/ab/old/conv_tiles_pre.json; else L=$PWD/rdeic_amd/lib/librdeic_hip.so; TT=$PWD/rdeic_amd/conv_tiles.json; fi
    RDEIC_LIB=$L RDEIC_TILE_TABLE=$TT timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --fp32-steps 0 > $O/$T$i.json 2> $O/$T$i.err || { echo "bench $T$i failed"; tail -5 $O/$T$i.err; exit 7; }
    python3 -c "import json; d=json.loads(open('$O/$T$i.json').read().strip().splitlines()[-1]); print('$T$i', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
