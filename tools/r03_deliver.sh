# Round-3 measurement deliverables (one GPU call): config-4 bpp sweep line, config-3 line, rocprof
# kernel trace of the bench (step slice), PMC conv traffic.
T=${1:-r03_deliver}
O=$PWD/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u bench.py --bpp-sweep 0.04,0.08,0.12 --no-cpu-baseline > $O/bpp_sweep.json 2> $O/bpp_sweep.err || { echo "sweep failed"; tail -5 $O/bpp_sweep.err; exit 1; }
echo "sweep ok"
timeout -k 10 600 python -u bench.py --size 1024 --ddim-steps 5 --batch 8 --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/config3.json 2> $O/config3.err || { echo "config3 failed"; tail -5 $O/config3.err; exit 1; }
echo "config3 ok"
bash tools/prof_layers.sh $T || exit 1
bash tools/pmc_bench.sh ${T}_pmc || exit 1
