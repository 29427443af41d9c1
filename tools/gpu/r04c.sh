#!/bin/bash
# r04: halo main-loop attribution (diagnostic builds: 1 no DMA waits, 2 no barriers, 3 both, 4 no MFMA,
# 8 no GroupNorm transform) + halo tests + stage-wise bf16-vs-fp32 values
set -o pipefail
O=gpurun_out/r04c
mkdir -p $O
for d in 0 1 2 3 4 8; do
  for cfg in "16 512 512 128 128 1 1" "16 128 128 512 512 1 1"; do
    echo -n "{\"diag\": $d, \"r\": " >> $O/halo_diag.jsonl
    timeout -k 5 60 tools/halo_stamps_d$d $cfg >> $O/halo_diag.jsonl 2>> $O/halo_diag.err || { echo "stamps d$d failed"; exit 3; }
    sed -i '$ s/$/}/' $O/halo_diag.jsonl
  done
done
cat $O/halo_diag.jsonl
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_halo_conv_gpu.py \
  tests/test_bf16_vs_fp32_gpu.py > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "bf16 vs fp32|passed|failed" $O/pytest.log | tail -5
exit $rc
