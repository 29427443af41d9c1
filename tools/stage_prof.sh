# rocprofv3 kernel stats per pipeline stage (run from the repo root on the GPU box)
set -e
R=$PWD
mkdir -p gpurun_out/stage
cd /tmp && export TMPDIR=/tmp
for st in unet vae_dec vae_enc; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/stage/$st -o s -- python3 $R/tools/stage_only.py --stage $st > $R/gpurun_out/stage/$st.log 2>&1
done
