#!/bin/bash
# SQ counters of the halo conv (tools/halo_stamps_cur: halo8, and halo4 via HALO4=1) on two VAE shapes:
# where do the waves of the main loop wait (barrier / vmcnt / LDS issue), how busy is the MFMA pipe,
# how many LDS bank-conflict cycles.
set -o pipefail
# usage (repo root on the box): bash tools/pmc_halo.sh TAG
R=$PWD
O=$R/gpurun_out/${1:-pmc_halo}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU"
for v in 8 4; do
  for cfg in "16 512 512 128 128 1 1" "16 256 256 256 256 1 1"; do
    tag=h${v}_$(echo $cfg | cut -d' ' -f2,4 | tr ' ' '_')
    i=1
    for P in "$P1" "$P2"; do
      HALO4=$([ $v = 4 ] && echo 1 || echo 0) timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/$tag/p$i -o p -- $R/tools/halo_stamps_cur $cfg > $O/$tag.p$i.log 2>&1 || { echo "$tag pass $i failed"; tail -5 $O/$tag.p$i.log; exit 1; }
      i=$((i+1))
    done
    echo "$tag ok"
  done
done
cd $R && python3 - "$O" <<'PY'
import csv, glob, sys, collections, json, os
o = sys.argv[1]
out = {}
for d in sorted(glob.glob(o + "/h*_*")):
    if not os.path.isdir(d): continue
    agg = collections.defaultdict(float); n = collections.Counter()
    for path in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if "halo" not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    avg = {c: agg[c] / n[c] for c in agg}
    wc = avg.get("SQ_WAVE_CYCLES", 1)
    out[os.path.basename(d)] = {"per_launch": {c: round(v) for c, v in sorted(avg.items())},
        "frac_of_wave_cycles": {c: round(avg[c] / wc, 4) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM") if c in avg},
        "lds_conflict_over_active": round(avg.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, avg.get("SQ_LDS_IDX_ACTIVE", 1)), 4)}
json.dump(out, open(o + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
