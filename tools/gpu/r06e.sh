#!/bin/bash
# r06: edge-conv / fused-GroupNorm micro A/B and their tests.
set -o pipefail
TAG=${1:-r06e}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -u tools/edge_bench.py 20 > $O/edge_bench.jsonl 2> $O/edge_bench.err || { echo "edge bench failed"; tail -20 $O/edge_bench.err; exit 3; }
cat $O/edge_bench.jsonl
timeout -k 10 600 python3 -u -m pytest tests/test_edge_convs_gpu.py tests/test_gn_fused_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
