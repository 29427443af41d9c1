#!/bin/bash
# r04: halo tests on the HSPLIT/TW4/VMFAST library; S3/S4 ring tiles (39-41) on the transformer linears
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_halo_conv_gpu.py > $O/pytest_halo.log 2>&1 || { echo "halo tests failed"; tail -30 $O/pytest_halo.log; exit 4; }
tail -1 $O/pytest_halo.log
timeout -k 10 400 python -u tools/lin_bench.py > $O/lin.jsonl 2> $O/lin.err || { echo "lin_bench failed"; tail -20 $O/lin.err; exit 3; }
cat $O/lin.jsonl
