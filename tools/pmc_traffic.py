"""Aggregate the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_bench.sh into HBM bytes per conv
launch (rdeic conv kernels: conv_dma_kernel, conv_kernel, conv3x3_smallc, splitk_reduce; not the
weight packing). gfx950: FETCH_SIZE counts half the bytes of wide streaming reads
(MI355X_MICROARCH.md §HBM), so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. Only the dispatches
of the timed bench step count: those after the warm-up step's image_mse kernel."""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(pattern, counter):
    rows = []
    for path in glob.glob(pattern, recursive=True):
        rows += [r for r in csv.DictReader(open(path)) if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if "image_mse" in r["Kernel_Name"]]
    rows = rows[marks[-2] + 1:marks[-1] + 1] if len(marks) >= 2 else rows
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    vgpr = {}
    for r in rows:
        name = r["Kernel_Name"]
        if ("conv" not in name and "splitk_reduce" not in name) or "pack_conv" in name:
            continue
        tot[name] += float(r["Counter_Value"])
        cnt[name] += 1
        vgpr[name] = (int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]))
    return tot, cnt, vgpr


def workload(argv):
    """The bench workload the passes ran (bench.py's defaults overridden by the args pmc_bench.sh
    forwarded): bench.py attaches the traffic only to a line of the same workload."""
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--ddim-steps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--sampler", default="ddim")
    a, _ = ap.parse_known_args(argv)
    return {"size": a.size, "ddim_steps": a.ddim_steps, "batch": a.batch, "dtype": a.dtype, "sampler": a.sampler}


out_dir = sys.argv[1]
f_tot, f_cnt, vgpr = per_kernel(os.path.join(out_dir, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE")
w_tot, w_cnt, _ = per_kernel(os.path.join(out_dir, "write", "**", "*counter_collection.csv"), "WRITE_SIZE")
launches = sum(f_cnt.values())
fetch_b = 2 * sum(f_tot.values()) * 1024
write_b = sum(w_tot.values()) * 1024
red = [k for k in f_tot if "splitk_reduce" in k]
red_b = sum(2 * f_tot[k] * 1024 + w_tot.get(k, 0) * 1024 for k in red)
print(json.dumps({
    # per step (the one timed bench step the passes cover): the figure bench.py divides by the library's
    # algorithmic bytes of the same step (both cover every conv launch of the step; the split-K reduce
    # launches have no algorithmic bytes of their own and are also reported apart)
    "bytes_per_step": round(fetch_b + write_b),
    "splitk_reduce_bytes_per_step": round(red_b),
    "splitk_reduce_launches": sum(f_cnt[k] for k in red),
    "bytes_per_launch": round((fetch_b / max(1, launches)) + write_b / max(1, sum(w_cnt.values()))),
    "fetch_bytes_per_launch": round(fetch_b / max(1, launches)),
    "write_bytes_per_launch": round(write_b / max(1, sum(w_cnt.values()))),
    "launches_counted": launches,
    "head": os.environ.get("RDEIC_HEAD"),  # the commit the passes ran (set by the GPU round script)
    "workload": workload(sys.argv[2:]),
    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 1 --warmup 1, timed step only "
              "(tools/pmc_bench.sh)",
    "per_kernel": {k[:80]: {"launches": f_cnt[k], "gb": round((2 * f_tot[k] * 1024 + w_tot.get(k, 0) * 1024) / 1e9, 3),
                            "vgpr_agpr_lds": vgpr[k]} for k in f_tot},
}, indent=1))
