#!/bin/bash
# r04 first GPU pass: new parity tests + the --gpus launcher rehearsal (2 ranks sharing the GPU over gloo)
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
for cfg in "16 512 512 128 128 1 1" "16 512 512 128 128 0 0" "16 512 512 128 128 1 0" "16 512 512 128 128 0 1" \
           "16 256 256 256 256 1 1" "16 128 128 512 512 1 1"; do
  timeout -k 5 60 tools/halo_stamps $cfg >> $O/halo_stamps.jsonl 2>> $O/halo_stamps.err || { echo "halo_stamps failed"; exit 3; }
done
cat $O/halo_stamps.jsonl
timeout -k 10 1200 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_halo_conv_gpu.py tests/test_config3_gpu.py::test_config3_fp32_noise_estimator_vs_reference \
  tests/test_bf16_vs_fp32_gpu.py tests/test_finetune_gpu.py tests/test_sessions_gpu.py "tests/test_kernels_gpu.py::test_layernorm_folded_linear" > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
RDEIC_LAUNCH_SHARE_GPU=1 timeout -k 10 420 python -u bench.py --gpus 2 --steps 4 --warmup 1 --streams 2 --no-cpu-baseline \
  > $O/bench_gpus2_shared.json 2> $O/bench_gpus2_shared.err
echo "bench2 rc=$?"
tail -c 600 $O/bench_gpus2_shared.json
