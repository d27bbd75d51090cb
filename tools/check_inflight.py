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
  * an asm load (or an asm atomic with return, sc0) adds its destination
    registers at age 0;
  * `s_waitcnt vmcnt(N)` (asm or compiler) retires entries of age >= N;
  * ages are capped at 64 (vmcnt holds at most 63 outstanding operations);
  * at a join the states are merged keeping each register's youngest age;
  * short branch-only blocks that test a constant SGPR pair / vcc are walked
    per incoming edge, so a branch decided by a constant prunes its dead edge.

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
    # an asm atomic with return (sc0) lands in its destination like a load
    ret = asm and is_vmem and ("load" in op or ("atomic" in op and re.search(r"\bsc0\b", t) is not None))
    if report is not None and not (ret and not (srcs & set(state))):
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
        if ret:
            for r in dst:
                state[r] = 0
    return state


def merge(a, b):
    out = dict(a)
    for r, x in b.items():
        out[r] = min(out.get(r, 64), x)
    return out


SREG = re.compile(r"^s\[(\d+):(\d+)\]$|^s(\d+)$")


def sregs(tok):
    m = SREG.match(tok.strip())
    if not m:
        return {"vcc"} if tok.strip().startswith("vcc") else set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def cstep(consts, t):
    """Constant SGPR-pair / vcc values through one instruction: enough to see
    hipcc's loop-exit funnel (s_mov_b64 X, 0 ... s_xor_b64 X, X, -1;
    s_andn2_b64 vcc, exec, X; s_cbranch_vccz) as the branch it always is."""
    parts = t.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    c = dict(consts)
    if op == "s_mov_b64" and len(ops) == 2 and ops[1] in ("0", "-1"):
        dst = ops[0]
        c = {k: v for k, v in c.items() if not (sregs(k) & sregs(dst))}
        c[dst] = int(ops[1])
        return c
    if op == "s_xor_b64" and len(ops) == 3 and ops[2] == "-1" and ops[1] in c:
        v = ~c[ops[1]]
        c = {k: x for k, x in c.items() if not (sregs(k) & sregs(ops[0]))}
        c[ops[0]] = v
        return c
    if op == "s_mov_b64" and len(ops) == 2 and ops[1] in c:
        v = c[ops[1]]
        c = {k: x for k, x in c.items() if not (sregs(k) & sregs(ops[0]))}
        c[ops[0]] = v
        return c
    if op in ("s_andn2_b64", "s_and_b64") and len(ops) == 3 and ops[0] == "vcc" and ops[1] == "exec":
        x = c.get(ops[2])
        c.pop("vcc", None)
        if x is not None:  # exec is non-zero in a running wave
            zero = (x == -1) if op == "s_andn2_b64" else (x == 0)
            c["vcc"] = 0 if zero else 1
        return c
    written = set()
    if ops and (op.startswith("s_") or op.startswith("v_readlane") or op.startswith("v_readfirstlane")):
        written = sregs(ops[0])
    if op.startswith(("v_cmp", "v_add_co", "v_sub_co", "v_subrev_co", "v_addc", "v_subb", "v_div_scale")) or \
            (ops and ops[0].startswith("vcc")):
        written |= {"vcc"}
    if written:
        c = {k: v for k, v in c.items() if not (sregs(k) & written)}
    return c


def feasible(insts, bl, succ, n, consts):
    """Successors of block n, dropping a vccz/vccnz edge that vcc rules out."""
    a, b = bl[n]
    t = insts[b - 1][1]
    op = t.split()[0]
    if op not in ("s_cbranch_vccz", "s_cbranch_vccnz") or "vcc" not in consts or len(succ[n]) != 2:
        return succ[n]
    taken = (consts["vcc"] == 0) == (op == "s_cbranch_vccz")
    return [succ[n][0]] if taken else [succ[n][1]]


def cmerge(a, b):
    return {k: v for k, v in a.items() if b.get(k) == v}


def main():
    insts, labels = parse(sys.argv[1])
    bl, succ = blocks(insts, labels)
    ins = [None] * len(bl)
    cin = [None] * len(bl)

    def is_threadable(n):
        # short blocks without vector-memory ops or waits: hipcc's exit funnels
        # (a vcc branch on a constant SGPR pair) and the one- or two-
        # instruction blocks that lead into them (copies, then fall-through),
        # so a constant set on one path survives to the branch that tests it
        a, b = bl[n]
        if b - a > 8:
            return False
        return not any(insts[k][1].split()[0].startswith(VMEM) or insts[k][1].startswith("s_waitcnt")
                       for k in range(a, b))

    threadable = [n != 0 and is_threadable(n) for n in range(len(bl))]
    ins[0] = {}
    cin[0] = {}
    work = [0]
    while work:
        n = work.pop()
        st = dict(ins[n])
        cs = dict(cin[n])
        a, b = bl[n]
        for k in range(a, b):
            st = step(st, insts[k])
            cs = cstep(cs, insts[k][1])
        # Jump threading: a block with no vector-memory op or wait that ends in
        # a vcc branch (the funnel) is walked per incoming edge, so a constant
        # known on one edge is not lost in the merge with the others.
        edges = [(s, cs) for s in feasible(insts, bl, succ, n, cs)]
        hops = 0
        while edges:
            s, c = edges.pop()
            if threadable[s] and hops < 64:
                hops += 1
                ins[s] = st if ins[s] is None else merge(ins[s], st)  # for the report pass
                c2 = c
                for k in range(bl[s][0], bl[s][1]):
                    c2 = cstep(c2, insts[k][1])
                edges.extend((t, c2) for t in feasible(insts, bl, succ, s, c2))
                continue
            new = st if ins[s] is None else merge(ins[s], st)
            newc = c if cin[s] is None else cmerge(cin[s], c)
            if new != ins[s] or newc != cin[s]:
                ins[s] = new
                cin[s] = newc
                work.append(s)
    # Joins keep each register's youngest age.  hipcc funnels loop exits through
    # a block that tests a constant-set SGPR pair (s_mov_b64 X, 0 ... s_xor_b64
    # X, X, -1; s_andn2_b64 vcc, exec, X; s_cbranch_vccz) and also falls into
    # the loop header; walking such blocks per incoming edge (jump threading
    # above) drops those infeasible paths, which used to carry young loads into
    # the header by the hundreds.  What is left is counted in two classes, and
    # BOTH fail the audit: a touch placed before an asm vmcnt wait in its own
    # block (the compiler materialising a ring register for the wait's "+v"
    # operand from a stale copy), and any other touch.
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
    for ln, t, regs in possible[:40]:
        print(f"line {ln}: {t}   in-flight {regs}")
    print(f"{len(certain)} hazards before a wait; {len(possible)} other hazards ({len(bl)} blocks)")
    return 1 if certain or possible else 0


if __name__ == "__main__":
    sys.exit(main())
