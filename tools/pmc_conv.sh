# PMC passes over single conv shapes (each pass its own rocprofv3 run; SQ <= 8, TCC <= 4 counters)
# usage: bash tools/pmc_conv.sh "vae128@512 vae512@128"
set -e
R=$PWD
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for shape in ${1:-vae128@512 vae512@128}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/pmc/a_$shape -o p -- python3 $R/tools/conv_one.py --shape $shape --paths 2 > $R/gpurun_out/pmc/a_$shape.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc/b_$shape -o p -- python3 $R/tools/conv_one.py --shape $shape --paths 2 > $R/gpurun_out/pmc/b_$shape.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc/c_$shape -o p -- python3 $R/tools/conv_one.py --shape $shape --paths 2 > $R/gpurun_out/pmc/c_$shape.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc/d_$shape -o p -- python3 $R/tools/conv_one.py --shape $shape --paths 2 > $R/gpurun_out/pmc/d_$shape.log 2>&1
done
