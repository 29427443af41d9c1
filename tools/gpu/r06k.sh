#!/bin/bash
# r06: halo8 transposed-MFMA / register epilogue: halo + config-2 tests, then a same-box stamps A/B (old vs cur)
set -o pipefail
TAG=${1:-r06k}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_halo_conv_gpu.py tests/test_config2_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 4; }
grep -E "passed|failed" $O/pytest.log | tail -1
HALO_AB_SHAPES=${HALO_AB_SHAPES:-"16,512,512,128,128 16,256,256,256,256 16,128,128,512,512 16,512,512,256,128"} bash tools/gpu/halo_ab.sh $TAG 2 ${HALO_AB_VARIANTS:-old:old cur:cur}
