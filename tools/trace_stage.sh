# kernel trace of one pipeline stage for gap analysis
set -e
R=$PWD
mkdir -p gpurun_out/trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace/$1 -o t -- python3 $R/tools/stage_only.py --stage $1 --reps 3 > $R/gpurun_out/trace/$1.log 2>&1
