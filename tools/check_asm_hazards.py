#!/usr/bin/env python3
"""Audit a gfx950 .s for VALU-written SGPRs read by inline-asm VMEM within 5
wait states (cdna_hip_programming.md 5.7 item 2): prints suspicious sites."""
import re
import sys

def sregs(tok):
    m = re.match(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", tok)
    return {int(m.group(1))} if m else set()

lines = open(sys.argv[1]).read().splitlines()
bad = 0
for i, l in enumerate(lines):
    t = l.strip()
    if not (t.startswith("global_load") or t.startswith("buffer_load")):
        continue
    if i == 0 or "ASMSTART" not in lines[i - 1]:
        continue
    ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
    read = set()
    for o in ops[1:]:
        read |= sregs(o.split()[0])
    # walk back over real instructions counting wait states
    states, j = 0, i - 1
    while j >= 0 and states < 6:
        u = lines[j].strip()
        j -= 1
        if not u or u.startswith(";") or u.startswith(".") or u.endswith(":"):
            continue
        if u.startswith("s_nop"):
            states += int(u.split()[1]) + 1
            continue
        parts = u.split(None, 1)
        if parts[0].startswith("v_") and len(parts) > 1:
            dst = parts[1].split(",")[0].strip()
            if sregs(dst) & read:
                print(f"line {i+1}: {t}  <- {u} ({states} states before)")
                bad += 1
        states += 1
print(f"{bad} suspicious sites")


def vregs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


# Second audit: registers written by inline-asm loads that the compiler touches
# (reads, copies, overwrites) before an inline-asm s_waitcnt vmcnt retires them.
pending = {}
touch = 0
for i, l in enumerate(lines):
    t = l.strip()
    if not t or t.startswith(";") or t.endswith(":") or t.startswith("."):
        continue
    asm = i > 0 and "ASMSTART" in lines[i - 1]
    if asm and t.startswith("s_waitcnt") and "vmcnt" in t:
        pending.clear()
        continue
    if t.startswith("s_endpgm") or t.startswith("s_branch") or t.startswith("s_cbranch"):
        continue
    parts = t.split(None, 1)
    ops = [o.strip().split()[0] for o in parts[1].split(",")] if len(parts) > 1 else []
    regs = set()
    for o in ops:
        regs |= vregs(o)
    if asm and (parts[0].startswith("global_load") or parts[0].startswith("buffer_load")):
        for r in vregs(ops[0]):
            pending[r] = i
        continue
    srcs = set()
    for o in ops[1:]:
        srcs |= vregs(o)
    # stores/DS ops read their first operand too; VALU dests are ops[0]
    if parts[0].startswith(("global_store", "buffer_store", "ds_write", "v_readlane", "v_readfirstlane")):
        srcs |= vregs(ops[0]) if ops else set()
    hit = srcs & set(pending)
    if hit:
        touch += 1
        if touch <= 20:
            print(f"line {i+1}: {t}   touches pending {sorted(hit)}")
print(f"{touch} reads of in-flight asm-load registers (linear scan, may include other-branch false positives)")

sys.exit(1 if bad else 0)
