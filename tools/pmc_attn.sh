# PMC passes over one attention shape (each pass its own rocprofv3 run)
# usage: bash tools/pmc_attn.sh SHAPE OUTDIR
set -e
R=$PWD
S=${1:-self4096}; O=$R/gpurun_out/${2:-pmc_attn}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/a -o p -- python3 $R/tools/attn_one.py --shape $S > $O/a.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/b -o p -- python3 $R/tools/attn_one.py --shape $S > $O/b.log 2>&1
echo done
