# HBM traffic of the bench's conv launches from PMC counters: two separate rocprofv3 --pmc passes
# over a short bench run (FETCH_SIZE; WRITE_SIZE — they do not fit one pass), then
# tools/pmc_traffic.py -> <out>/conv_traffic.json (FETCH_SIZE x 2 + WRITE_SIZE per launch, KB -> B).
# usage (repo root on the GPU box): bash tools/pmc_bench.sh TAG [bench args, e.g. --size 1024 --ddim-steps 5 --batch 8]
set -e
R=$PWD
O=$R/gpurun_out/${1:-pmc_bench}
shift || true
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- python3 $R/bench.py --steps 1 --warmup 1 --streams 1 --no-cpu-baseline --no-roofline --fp32-steps 0 "$@" > $O/fetch.log 2>&1
echo "fetch pass ok"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- python3 $R/bench.py --steps 1 --warmup 1 --streams 1 --no-cpu-baseline --no-roofline --fp32-steps 0 "$@" > $O/write.log 2>&1
echo "write pass ok"
cd $R && python3 tools/pmc_traffic.py $O "$@" > $O/conv_traffic.json && cat $O/conv_traffic.json
