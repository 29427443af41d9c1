#!/bin/bash
# r04: halo epilogue v2 (4 passes, residual by LDS-DMA one pass ahead) — stamps, halo tests, and the
# measured bf16-vs-fp32 stage bounds (printed with -s)
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
for cfg in "16 512 512 128 128 1 1" "16 512 512 128 128 0 0" "16 512 512 128 128 1 0" \
           "16 256 256 256 256 1 1" "16 128 128 512 512 1 1" "16 64 64 512 512 1 1"; do
  timeout -k 5 60 tools/halo_stamps $cfg >> $O/halo_stamps.jsonl 2>> $O/halo_stamps.err || { echo "halo_stamps failed"; exit 3; }
done
cat $O/halo_stamps.jsonl
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_halo_conv_gpu.py \
  tests/test_bf16_vs_fp32_gpu.py tests/test_gn_fused_gpu.py "tests/test_finetune_gpu.py::test_gradients_of_every_trainable_tensor" \
  > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "bf16 vs fp32|passed|failed" $O/pytest.log | tail -5
exit $rc
