#!/bin/bash
# A/B of two library builds on the attention kernels: parity tests on the new build, then
# tools/attn_bench.py on each (interleaved). usage: bash tools/gpu/attn_ab.sh TAG LIB_OLD [REPS]
set -o pipefail
O=$PWD/gpurun_out/${1:-attn_ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k attention > $O/pytest_attn.log 2>&1 || { echo "attention tests failed"; tail -30 $O/pytest_attn.log; exit 4; }
tail -1 $O/pytest_attn.log
for rep in $(seq 1 ${3:-2}); do
  for v in old new; do
    L=$PWD/rdeic_amd/lib/librdeic_hip.so; [ $v = old ] && L=$PWD/$2
    RDEIC_LIB=$L timeout -k 10 300 python -u tools/attn_bench.py > $O/attn_${v}_$rep.txt 2>&1 || { echo "attn_bench $v failed"; tail -5 $O/attn_${v}_$rep.txt; exit 3; }
    echo "== $v $rep"; grep -v amdgpu.ids $O/attn_${v}_$rep.txt | grep ctrl16
  done
done
