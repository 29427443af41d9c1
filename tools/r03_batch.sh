# halo tests + A/B, config-3 sequence probe, per-layer profile (one GPU call)
T=${1:-r03e}
bash tools/halo_check.sh $T || exit $?
O=$PWD/gpurun_out/$T
timeout -k 10 400 python -u tools/probe/c3_sequence.py > $O/c3seq.txt 2>&1
rc=$?; tail -12 $O/c3seq.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/prof_layers.sh $T
