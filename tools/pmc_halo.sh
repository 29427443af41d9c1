# PMC passes over tools/halo_one.py (halo kernel vs im2col tile on one VAE shape)
# usage (repo root on the box): bash tools/pmc_halo.sh TAG [H cin cout]
R=$PWD
O=$R/gpurun_out/${1:-pmc_halo}
shift || true
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/p$i -o p -- python3 $R/tools/halo_one.py "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  echo "pass $i ok"
  i=$((i+1))
done
cd $R && python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for path in glob.glob(o + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "conv" not in k: continue
        name = "halo" if "halo" in k else ("dma" if "dma" in k else k[:40])
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
for name, d in agg.items():
    print(name, {c: round(v / 1e6, 3) for c, v in sorted(d.items())})
PY
