# halo conv GPU tests + A/B bench + config-3 determinism probe (one GPU call)
# usage (repo root on the box): bash tools/halo_check.sh TAG
O=$PWD/gpurun_out/${1:-halo}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_halo_conv_gpu.py -v --timeout 120 --timeout-method thread > $O/halo_test.log 2>&1
rc=$?; tail -15 $O/halo_test.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/halo_bench.py > $O/halo_bench.txt 2>&1
rc=$?; tail -12 $O/halo_bench.txt
if [ $rc -ne 0 ]; then exit $rc; fi
