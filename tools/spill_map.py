"""Where does a kernel spill? Compiles one HIP source to gfx950 assembly and prints, for one kernel (substring of
its mangled name), the scratch instructions with their position relative to the MFMA range (main loop).
usage: python tools/spill_map.py SRC.hip NAME_SUBSTR [extra hipcc flags...]"""
import os
import re
import subprocess
import sys
import tempfile


def main():
    src, pat, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = os.path.join(tempfile.gettempdir(), "spill_map.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", src,
                    "-o", out] + extra, check=True, stderr=subprocess.DEVNULL)
    s = open(out).read()
    for name in sorted(set(re.findall(r"^(_Z\w*" + re.escape(pat) + r"\w*):", s, re.M))):
        body = s[s.index(name + ":"):s.index(".Lfunc_end", s.index(name + ":"))].splitlines()
        m = [i for i, l in enumerate(body) if "v_mfma" in l]
        sc = [(i, l.strip()) for i, l in enumerate(body) if "scratch_" in l]
        lo, hi = (m[0], m[-1]) if m else (0, 0)
        inside = sum(1 for i, _ in sc if lo <= i <= hi)
        print(f"{name}: {len(body)} lines, mfma {len(m)} in [{lo}, {hi}], scratch ops {len(sc)} ({inside} inside the mfma range)")
        for i, l in sc:
            print(f"  {i:6d} {'IN ' if lo <= i <= hi else '   '} {l}")


if __name__ == "__main__":
    main()
