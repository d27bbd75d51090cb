#!/usr/bin/env python3
"""CFG-aware audit of inline-asm prefetch rings in a gfx950 kernel (.s).

The ring's loads are inline asm, so the compiler does not know their VGPRs are
still being written by the memory system until the asm `s_waitcnt vmcnt(N)`
that retires them.  Any compiler-generated read, copy or overwrite of such a
register before that wait is a real hazard (stale data or a clobbered result).
This walks the kernel's control-flow graph (labels, s_branch, s_cbranch_*,
fall-through) with a forward dataflow over "possibly in-flight" registers:

  * every vector-memory instruction (asm or not, loads and stores: they share
    vmcnt) ages the in-flight entries by one;
  * an asm load adds its destination registers at age 0;
  * `s_waitcnt vmcnt(N)` (asm or compiler) retires entries of age >= N;
  * ages are capped at 64 (vmcnt holds at most 63 outstanding operations);
  * at a join the states are merged keeping each register's youngest age.

Usage: check_inflight.py kernel.s   (the text of ONE kernel, e.g. cut with awk)
Exit status 1 if any hazard is found.
"""
import re
import sys

VMEM = ("global_", "buffer_", "flat_", "scratch_")


def vregs(tok):
    tok = tok.strip()
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def parse(path):
    lines = open(path).read().splitlines()
    insts = []  # (lineno, text, is_asm)
    labels = {}
    in_asm = False
    for i, l in enumerate(lines):
        t = l.split(";")[0].strip() if not l.strip().startswith(";;#ASM") else l.strip()
        if l.strip() == ";;#ASMSTART":
            in_asm = True
            continue
        if l.strip() == ";;#ASMEND":
            in_asm = False
            continue
        if t.endswith(":"):
            labels[t[:-1]] = len(insts)
            continue
        if not t or t.startswith("."):
            continue
        insts.append((i + 1, t, in_asm))
    return insts, labels


def blocks(insts, labels):
    starts = {0} | set(labels.values())
    for k, (_, t, _) in enumerate(insts):
        op = t.split()[0]
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op == "s_endpgm" or op.startswith("s_setpc"):
            starts.add(k + 1)
    starts = sorted(s for s in starts if s <= len(insts))
    bl = []
    for a, b in zip(starts, starts[1:] + [len(insts)]):
        if a < b:
            bl.append((a, b))
    idx = {a: n for n, (a, _) in enumerate(bl)}
    succ = []
    for n, (a, b) in enumerate(bl):
        t = insts[b - 1][1]
        op = t.split()[0]
        s = []
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            tgt = t.split()[1]
            if tgt in labels and labels[tgt] in idx:
                s.append(idx[labels[tgt]])
        if not (op.startswith("s_branch") or op == "s_endpgm" or op.startswith("s_setpc")):
            if b in idx:
                s.append(idx[b])
        succ.append(s)
    return bl, succ


def step(state, inst, report=None):
    ln, t, asm = inst
    parts = t.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    if op == "s_waitcnt":
        m = re.search(r"vmcnt\((\d+)\)", t)
        if m:
            n = int(m.group(1))
            return {r: a for r, a in state.items() if a < n}
        return state
    is_vmem = op.startswith(VMEM)
    dst = vregs(ops[0].split()[0]) if ops else set()
    srcs = set()
    for o in ops[1:]:
        srcs |= vregs(o.split()[0])
    if op.startswith(("global_store", "buffer_store", "flat_store", "ds_write", "v_readlane", "v_readfirstlane",
                      "v_writelane")):
        srcs |= dst
        if not op.startswith("v_writelane"):
            dst = set()
    if report is not None and not (asm and is_vmem and op.find("load") >= 0 and not (srcs & set(state))):
        hit = (srcs | dst) & set(state)
        if hit:
            report.append((ln, t, sorted(hit)))
    elif report is not None and asm and is_vmem:
        hit = srcs & set(state)
        if hit:
            report.append((ln, t, sorted(hit)))
    if is_vmem:
        state = {r: min(a + 1, 64) for r, a in state.items()}
        state = {r: a for r, a in state.items() if a < 64}
        if asm and "load" in op:
            for r in dst:
                state[r] = 0
    return state


def merge(a, b):
    out = dict(a)
    for r, x in b.items():
        out[r] = min(out.get(r, 64), x)
    return out


def main():
    insts, labels = parse(sys.argv[1])
    bl, succ = blocks(insts, labels)
    ins = [None] * len(bl)
    ins[0] = {}
    work = [0]
    while work:
        n = work.pop()
        st = dict(ins[n])
        a, b = bl[n]
        for k in range(a, b):
            st = step(st, insts[k])
        for s in succ[n]:
            new = st if ins[s] is None else merge(ins[s], st)
            if new != ins[s]:
                ins[s] = new
                work.append(s)
    # The dataflow is path-insensitive: hipcc often funnels a loop exit through
    # a flag-tested block that also falls into the loop header, which makes
    # infeasible paths look like they carry young loads into the header.  So
    # the verdict counts only the unambiguous pattern -- a read/copy of a
    # possibly in-flight register placed BEFORE an asm vmcnt wait in the same
    # basic block (the compiler materialising a ring register for the wait's
    # "+v" operand from a stale copy) -- and reports the rest as "possible".
    certain, possible = [], []
    for n, (a, b) in enumerate(bl):
        if ins[n] is None:
            continue
        st = dict(ins[n])
        waits = [k for k in range(a, b) if insts[k][2] and insts[k][1].startswith("s_waitcnt")]
        last_wait = waits[-1] if waits else -1
        for k in range(a, b):
            rep = []
            st = step(st, insts[k], rep)
            (certain if k < last_wait else possible).extend(rep)
    for ln, t, regs in certain[:40]:
        print(f"line {ln}: {t}   in-flight {regs}  (before the asm wait of its block)")
    print(f"{len(certain)} hazards; {len(possible)} possible on path-insensitive joins ({len(bl)} blocks)")
    return 1 if certain else 0


if __name__ == "__main__":
    sys.exit(main())
