# Per-layer conv table of the bench workload (eager, Python-event timed) and a rocprofv3 kernel
# trace of a short bench run sliced to its last single-session step.
# usage (repo root on the box): bash tools/prof_layers.sh TAG
TAG=${1:-layers}
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pipeline_profile.py --top 120 > $O/layers.txt 2> $O/layers.err || { echo "pipeline_profile failed"; tail -5 $O/layers.err; exit 1; }
head -3 $O/layers.txt
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err || { echo "rocprof bench failed"; tail -5 $O/bench_prof.err; exit 1; }
cd $R
python tools/step_kernels.py $O/prof/bench_kernel_trace.csv --bench $O/bench_prof.json --out $O/step_kernels.json > /dev/null && echo "step summary ok"
