# PMC passes for one conv shape on given tiles (each pass its own rocprofv3 run)
# usage: bash tools/pmc_tiles.sh SHAPE "34 25" OUTDIR
set -e
R=$PWD
S=$1; TILES=$2; O=$R/gpurun_out/${3:-pmc_tiles}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for t in $TILES; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/a_$t -o p -- python3 $R/tools/conv_one.py --shape $S --paths 2 --tile $t --reps 5 > $O/a_$t.log 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $O/b_$t -o p -- python3 $R/tools/conv_one.py --shape $S --paths 2 --tile $t --reps 5 > $O/b_$t.log 2>&1
  echo "tile $t done"
done
