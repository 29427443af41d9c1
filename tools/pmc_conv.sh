set -e
R=$PWD
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for shape in vae128@512 vae512@128; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/pmc/a_$shape -o p -- python3 $R/tools/conv_one.py --shape $shape > $R/gpurun_out/pmc/a_$shape.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/pmc/b_$shape -o p -- python3 $R/tools/conv_one.py --shape $shape > $R/gpurun_out/pmc/b_$shape.log 2>&1
done
