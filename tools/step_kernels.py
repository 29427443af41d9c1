"""Slice a rocprofv3 kernel trace to the LAST timed bench step and summarise it per kernel family.

bench.py ends every step with exactly one `image_mse_kernel` launch, so the last step is the span
of dispatches after the second-to-last `image_mse_kernel` up to and including the last one. The
summary gives, per family and per kernel template: launches, busy ms, and for the step as a whole
its wall span, the kernel-busy time and the idle time (span - union of kernel intervals).

With --bench (the bench line printed by the SAME profiled run, which carries
roofline.flops_per_step), the conv family's algorithmic TFLOP/s and roofline fraction are
recomputed from the trace: frac = flops_per_step / trace conv ms / peak. That is the
cross-check profiles/README.md prescribes.

  python tools/step_kernels.py TRACE.csv [--bench bench_prof.json] [--out profiles/r02_step_kernels.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import subprocess
import sys

FAMILIES = [  # (family, substring on the demangled name), first match wins
    ("conv", "conv_dma_kernel"), ("conv", "conv_kernel"), ("conv", "conv3x3_smallc"), ("conv", "splitk_reduce"),
    ("conv", "conv3x3_halo"),
    ("conv", "conv_out_dot2"),
    ("attention", "attn"), ("vae_attention_softmax", "softmax_rows"),
    ("conv", "gn_narrow"), ("conv", "conv_in8"), ("groupnorm", "gn_"), ("layernorm", "layernorm"),
    ("entropy", "ckbd_"), ("entropy", "vq_argmin"), ("entropy", "gather_rows"), ("entropy", "row_sqnorm"),
    ("sampler", "ddim_step"), ("sampler", "spaced_step"), ("sampler", "axpby"), ("sampler", "cfg_combine"),
    ("image_io", "img_to_nhwc"), ("image_io", "nhwc_to_img"), ("image_io", "image_mse"),
    ("aten", "at::native"), ("copy", "rocclr"),
]


def _short_demangle(m: str) -> str:
    """Enough of the Itanium ABI for this library's kernels (binutils 2.38's c++filt does not know
    DF16b): `_ZN12_GLOBAL__N_1<len><name>I<args>E...` -> `name<args>`."""
    mm = re.match(r"_ZN12_GLOBAL__N_1(\d+)", m)
    if not mm:
        return m
    n = int(mm.group(1))
    rest = m[mm.end():]
    name, rest = rest[:n], rest[n:]
    if not rest.startswith("I"):
        return name
    args, i = [], 1
    while i < len(rest) and rest[i] != "E":
        for tok, val in (("DF16b", "__bf16"), ("f", "float"), ("i", "int")):
            if rest.startswith(tok, i):
                args.append(val)
                i += len(tok)
                break
        else:
            lit = re.match(r"L([ib])(\d+)E", rest[i:])
            if not lit:
                break
            v = lit.group(2)
            args.append(v if lit.group(1) == "i" else ("true" if v == "1" else "false"))
            i += lit.end()
    return f"{name}<{', '.join(args)}>"


def demangle(names):
    mangled = sorted({n for n in names if n.startswith("_Z")})
    out = {n: n for n in names}
    if mangled:
        try:
            r = subprocess.run(["c++filt"], input="\n".join(mangled), capture_output=True, text=True, check=True)
            for m, d in zip(mangled, r.stdout.splitlines()):
                out[m] = d
        except (OSError, subprocess.CalledProcessError):
            pass
    for m in mangled:
        if out[m].startswith("_Z"):
            out[m] = _short_demangle(m)
    return out


def template(name: str) -> str:
    """The kernel's template instantiation without its parameter list."""
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return name[:cut]


def family(name: str) -> str:
    for fam, key in FAMILIES:
        if key in name:
            return fam
    return "other"


def load(path):
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    dem = demangle([r[2] for r in rows])
    return [(s, e, dem[n]) for s, e, n in rows]


def last_step(rows):
    marks = [i for i, r in enumerate(rows) if "image_mse_kernel" in r[2]]
    if len(marks) < 2:
        raise SystemExit(f"need >= 2 image_mse_kernel launches to delimit a step, found {len(marks)}")
    return rows[marks[-2] + 1: marks[-1] + 1]


def summarise(step):
    span_ns = step[-1][1] - step[0][0]
    busy, cur_s, cur_e = 0, None, None  # union of kernel intervals
    for s, e, _ in step:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    fams, tmpl = {}, {}
    for s, e, n in step:
        f = family(n)
        a = fams.setdefault(f, [0, 0])
        a[0] += 1
        a[1] += e - s
        t = tmpl.setdefault((f, template(n)), [0, 0])
        t[0] += 1
        t[1] += e - s
    return {
        "launches": len(step), "span_ms": round(span_ns / 1e6, 3), "kernel_busy_ms": round(busy / 1e6, 3),
        "idle_ms": round((span_ns - busy) / 1e6, 3),
        "families": {f: {"launches": c, "ms": round(ns / 1e6, 3)}
                     for f, (c, ns) in sorted(fams.items(), key=lambda kv: -kv[1][1])},
        "templates": [{"family": f, "kernel": t, "launches": c, "ms": round(ns / 1e6, 3)}
                      for (f, t), (c, ns) in sorted(tmpl.items(), key=lambda kv: -kv[1][1])],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--bench", help="bench JSON line of the same profiled run")
    ap.add_argument("--out")
    a = ap.parse_args()
    import os
    summ = {"source": a.trace.split("gpurun_out/")[-1], "head": os.environ.get("RDEIC_HEAD"),
            "step": "last timed step (image_mse_kernel-delimited)"}
    summ.update(summarise(last_step(load(a.trace))))
    if a.bench:
        with open(a.bench) as f:
            line = json.loads([ln for ln in f if ln.startswith("{")][-1])
        roof = line["roofline"]
        fl = roof.get("flops_per_step")
        if fl:
            conv_ms = summ["families"]["conv"]["ms"]
            tf = fl / (conv_ms * 1e-3) / 1e12
            summ["conv_crosscheck"] = {
                "algorithmic_tflop_per_step": round(fl / 1e12, 3), "trace_conv_ms": conv_ms,
                "trace_tflops": round(tf, 1), "trace_frac": round(tf / roof["peak"], 4),
                "bench_line_frac": roof["frac"], "bench_line_conv_ms_per_step": roof["ms_per_step"]}
    js = json.dumps(summ, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")
    print(js)


if __name__ == "__main__":
    sys.exit(main())
