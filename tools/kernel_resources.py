"""Per-kernel register / LDS / scratch table of one HIP source, from the compiler's
-Rpass-analysis=kernel-resource-usage remarks (no GPU needed).

usage: python tools/kernel_resources.py SRC.hip [--filter SUBSTR] [--extra "-fno-slp-vectorize"] > table.txt
       python tools/kernel_resources.py --remarks FILE      (parse an existing remarks log)
"""
import argparse
import re
import subprocess
import sys


def parse(text):
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z \[\]/]+?): (\S+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    except Exception:
        return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="?")
    ap.add_argument("--remarks")
    ap.add_argument("--filter", default="")
    ap.add_argument("--extra", default="-fno-slp-vectorize")
    args = ap.parse_args()
    if args.remarks:
        text = open(args.remarks).read()
    else:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only", "-c",
               "-Rpass-analysis=kernel-resource-usage", args.src, "-o", "/dev/null"] + args.extra.split()
        text = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows = [r for r in parse(text) if args.filter in r["name"]]
    names = demangle([r["name"] for r in rows])
    print(f"{'SGPR':>5} {'VGPR':>5} {'AGPR':>5} {'scr':>4} {'occ':>3} {'LDS':>7}  kernel")
    for r, n in sorted(zip(rows, names), key=lambda x: x[1]):
        n = n.replace("(anonymous namespace)::", "").replace("__bf16", "bf16")
        print(f"{r.get('TotalSGPRs', '?'):>5} {r.get('VGPRs', '?'):>5} {r.get('AGPRs', '?'):>5} "
              f"{r.get('ScratchSize [bytes/lane]', '?'):>4} {r.get('Occupancy [waves/SIMD]', '?'):>3} "
              f"{r.get('LDS Size [bytes/block]', '?'):>7}  {n}")


if __name__ == "__main__":
    sys.exit(main())
