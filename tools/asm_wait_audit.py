"""Static audit of counted LDS waits in the compiled gfx950 ISA.

Inline-asm LDS reads (`ds_read_b64_tr_b16` in attention.hip, issued ahead and retired by a counted
`s_waitcnt lgkmcnt(N)`) are invisible to the compiler's own wait insertion, so the only guarantee
that a consumer reads the loaded registers after the data has landed is the ISA order. This tool
compiles a source file to gfx950 assembly (hipcc -S --cuda-device-only, the Makefile's flags), and
for every kernel runs a dataflow pass over its basic blocks:

  * each LDS-counter instruction (ds_*, s_load*/s_buffer_load*, s_sendmsg) enters a FIFO of
    outstanding operations with the registers it writes;
  * `s_waitcnt lgkmcnt(N)` retires the oldest entries until N remain (LDS returns in order);
  * an instruction that READS a register an outstanding entry still writes is a violation;
  * block entry states are the merge (union, aligned at the youngest end) of every predecessor's
    exit state, iterated to a fixpoint over the loop back edges.

Usage: python tools/asm_wait_audit.py rdeic_amd/csrc/attention.hip [--extra-flag ...]
Exit status 1 when any kernel has a violation; prints one line per kernel."""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REG = re.compile(r"\b([vas])(?:\[(\d+):(\d+)\]|(\d+)\b)")
LGKM_MAX = 15  # gfx9 lgkmcnt is 4 bits
WAIT = re.compile(r"lgkmcnt\((\d+)\)")
STORES = ("ds_write", "ds_store", "global_store", "buffer_store", "flat_store", "scratch_store", "ds_add",
          "global_atomic", "buffer_atomic")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        if kind == "s":
            continue  # scalar registers: SMEM results are checked the same way only for VGPR consumers
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(asm: str):
    """{kernel: [(label or None, mnemonic, operands)]} for every function in the file."""
    funcs, cur, name = {}, None, None
    for line in asm.splitlines():
        s = line.split(";")[0].rstrip()
        if not s.strip():
            continue
        if re.match(r"^[A-Za-z_.$][\w.$]*:", s):
            lab = s.split(":")[0]
            if not lab.startswith("."):
                name, cur = lab, []
                funcs[name] = cur
            elif cur is not None:
                if lab.startswith(".Lfunc_end"):
                    cur, name = None, None
                else:
                    cur.append((lab, None, ""))
            continue
        if cur is None or not s.startswith("\t") or s.strip().startswith("."):
            continue
        parts = s.strip().split(None, 1)
        cur.append((None, parts[0], parts[1] if len(parts) > 1 else ""))
    return funcs


def lgkm_op(mn: str) -> bool:
    return mn.startswith("ds_") or mn.startswith("s_load") or mn.startswith("s_buffer_load") or mn == "s_sendmsg"


def audit(ins):
    # basic blocks
    blocks, label_at = [], {}
    curb = []
    for it in ins:
        if it[0] is not None:
            if curb:
                blocks.append(curb)
            curb = []
            label_at[it[0]] = len(blocks)
            curb.append(it)
            continue
        curb.append(it)
        if it[1].startswith("s_branch") or it[1].startswith("s_cbranch") or it[1] == "s_endpgm" \
                or it[1].startswith("s_setpc"):
            blocks.append(curb)
            curb = []
    if curb:
        blocks.append(curb)
    succ = []
    for i, b in enumerate(blocks):
        last = b[-1]
        s = []
        if last[1] and (last[1].startswith("s_branch") or last[1].startswith("s_cbranch")):
            tgt = last[2].split()[0] if last[2] else ""
            if tgt in label_at:
                s.append(label_at[tgt])
        if not (last[1] and (last[1].startswith("s_branch") or last[1] == "s_endpgm")) and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)

    def merge(a, b):
        if a is None:
            return list(b)
        n = max(len(a), len(b))
        a2 = [frozenset()] * (n - len(a)) + list(a)
        b2 = [frozenset()] * (n - len(b)) + list(b)
        return [x | y for x, y in zip(a2, b2)]

    entry = [None] * len(blocks)
    entry[0] = []
    violations = {}
    work = [0]
    passes = 0
    while work and passes < 100000:
        passes += 1
        i = work.pop()
        q = list(entry[i])
        for lab, mn, ops in blocks[i]:
            if mn is None:
                continue
            if mn == "s_waitcnt" or mn == "s_waitcnt_lgkmcnt":
                m = WAIT.search(ops)
                if m:
                    keep = int(m.group(1))
                    while len(q) > keep:
                        q.pop(0)
                continue
            fields = [f.strip() for f in ops.split(",")] if ops else []
            if any(mn.startswith(p) for p in STORES):
                srcs = regs(ops)
                dsts = set()
            else:
                srcs = regs(",".join(fields[1:])) if fields else set()
                dsts = regs(fields[0]) if fields else set()
                if mn.startswith("v_mfma") and len(fields) >= 4:
                    srcs = regs(",".join(fields[1:4]))
            pending = set().union(*q) if q else set()
            hit = srcs & pending
            if hit:
                violations.setdefault((mn, ops), sorted(hit)[:4])
            if lgkm_op(mn):
                q.append(frozenset(d for d in dsts if d[0] in ("v", "a")))
                if len(q) > LGKM_MAX:  # the counter saturates: issue stalls until the oldest returns
                    q.pop(0)
        for j in succ[i]:
            new = merge(entry[j], q)
            if entry[j] is None or new != entry[j]:
                entry[j] = new
                work.append(j)
    return violations, len(blocks)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("source")
    ap.add_argument("--flags", default="", help="extra hipcc flags (the Makefile's per-file flags)")
    ap.add_argument("--kernel", default="", help="only kernels whose symbol contains this")
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
               args.source, "-o", out] + args.flags.split()
        subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
        asm = open(out).read()
    bad = 0
    for name, ins in parse(asm).items():
        if args.kernel not in name or not any(it[1] for it in ins):
            continue
        n_tr = sum(1 for it in ins if it[1] == "ds_read_b64_tr_b16")
        waits = sum(1 for it in ins if it[1] == "s_waitcnt" and "lgkmcnt" in it[2])
        v, nb = audit(ins)
        bad += bool(v)
        # negative control: with the counted (non-zero) lgkmcnt waits deleted, a kernel whose reads are
        # consumed through them must show violations, or the pass is not seeing its consumers
        stripped = [it for it in ins if not (it[1] == "s_waitcnt" and re.search(r"lgkmcnt\([1-9]", it[2] or ""))]
        ctrl = len(audit(stripped)[0]) if len(stripped) < len(ins) else 0
        print(f"{'VIOLATION' if v else 'ok':9s} {name}: {len(ins)} instr, {nb} blocks, {n_tr} ds_read_b64_tr_b16, "
              f"{waits} lgkmcnt waits, control without counted waits: {ctrl} violations"
              + (f"; first: {list(v.items())[:3]}" if v else ""))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
