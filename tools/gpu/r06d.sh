#!/bin/bash
# r06: edge-conv / fused-GroupNorm micro A/B, the focused tests, then the bench A/B against ab/r05.
set -o pipefail
TAG=${1:-r06d}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -u tools/edge_bench.py 20 > $O/edge_bench.jsonl 2> $O/edge_bench.err || { echo "edge bench failed"; tail -20 $O/edge_bench.err; exit 3; }
cat $O/edge_bench.jsonl
timeout -k 10 600 python3 -u -m pytest tests/test_edge_convs_gpu.py tests/test_gn_fused_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/new$i.json 2> $O/new$i.err || { echo "bench new failed"; tail -20 $O/new$i.err; exit 5; }
  python3 -c "import json;d=json.load(open('$O/new$i.json'));r=d['roofline'];print('new$i', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
  (cd ab/r05 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > $O/r05_$i.json 2> $O/r05_$i.err) || { echo "bench r05 failed"; tail -20 $O/r05_$i.err; exit 5; }
  python3 -c "import json;d=json.load(open('$O/r05_$i.json'));r=d['roofline'];print('r05_$i', d['value'], d['ms_per_step'], r['achieved'], r['frac'])"
done
