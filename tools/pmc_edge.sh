#!/bin/bash
# SQ counters of the VAE edge convs (tools/edge_bench.py only): where the waves of conv_in (ring) and the
# narrow norm -> SiLU -> conv_out wait, how busy VALU / MFMA / LDS are.
set -o pipefail
R=$PWD
O=$R/gpurun_out/${1:-pmc_edge}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $O/p$i -o p -- python3 $R/tools/edge_bench.py 3 only > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  i=$((i+1))
done
cd $R && python3 - "$O" <<'PY'
import csv, glob, sys, collections, json, os
o = sys.argv[1]
out = {}
for kname in ("conv_in8_ring_kernel", "conv3x3_gn_narrow_kernel"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for path in glob.glob(o + "/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(path)):
            if kname not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    avg = {c: agg[c] / n[c] for c in agg}
    wc = avg.get("SQ_WAVE_CYCLES", 1)
    out[kname] = {"per_launch": {c: round(v) for c, v in sorted(avg.items())},
        "frac_of_wave_cycles": {c: round(avg[c] / wc, 4) for c in avg if c.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_INST_CYCLES"))},
        "lds_conflict_over_active": round(avg.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, avg.get("SQ_LDS_IDX_ACTIVE", 1)), 4)}
json.dump(out, open(o + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
