# 160-wide tiles (37, 38) on the N = 320 layers: bit-identity on every layer shape, then TFLOP/s
# against the tiles the table uses. usage (repo root on the box): bash tools/n320_check.sh TAG
O=$PWD/gpurun_out/${1:-n320}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_tiles_gpu.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/dma_bench.py --tiles=-1,32,34,25,36,24,37,38 --reps 8 --only "320,x320" > $O/dma.jsonl 2> $O/dma.err; rc=$?
cat $O/dma.jsonl
exit $rc
