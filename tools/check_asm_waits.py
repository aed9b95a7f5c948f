#!/usr/bin/env python3
"""Static check of the counted-wait kernels (hand-placed `s_waitcnt vmcnt(N)` after inline-asm
loads, which the compiler's waitcnt pass does not track): walks the gfx950 assembly of each
named kernel in program order, models the vector-memory counter (loads + stores in issue
order) over the control-flow graph to a fixed point (paths merged conservatively, aligned
at the newest operation), and reports any instruction that reads or overwrites a load's
destination registers before a wait has retired that load on every path.

Usage: check_asm_waits.py file.s kernel_regex [...]   (exit 1 on a finding)"""
import re
import sys

VMEM = re.compile(r"^(global_load|global_store|buffer_load|buffer_store|global_atomic|buffer_atomic)\w*")


def regs(text):
    out = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        out |= set(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", text):
        out.add(int(a))
    return out


def blocks_of(lines):
    """basic blocks: (label, [instructions], [successor labels])"""
    blocks, cur, lab = [], [], "entry"
    nsplit = 0
    for raw in lines:
        t = raw.split(";")[0].strip()
        if not t:
            continue
        m = re.match(r"^(\.LBB\w+):", t)
        if m:
            blocks.append([lab, cur, None])
            lab, cur = m.group(1), []
            continue
        if t.startswith(".") or t.endswith(":"):
            continue
        cur.append(t)
        if t.startswith(("s_cbranch", "s_branch", "s_endpgm")):
            # a block ends at its branch: the target sees the state at the branch
            blocks.append([lab, cur, None])
            nsplit += 1
            lab, cur = "split%d" % nsplit, []
    blocks.append([lab, cur, None])
    order = [b[0] for b in blocks]
    for n, b in enumerate(blocks):
        succ = []
        ins = b[1]
        fall = True
        for t in ins:
            m = re.match(r"s_cbranch_\w+\s+(\.LBB\w+)", t)
            if m:
                succ.append(m.group(1))
            m = re.match(r"s_branch\s+(\.LBB\w+)", t)
            if m:
                succ.append(m.group(1))
                fall = False
            if t.startswith("s_endpgm"):
                fall = False
        if fall and n + 1 < len(blocks):
            succ.append(order[n + 1])
        b[2] = succ
    return {b[0]: b for b in blocks}, order


def merge(a, b):
    """outstanding VM ops (oldest first) of two paths, aligned at the newest"""
    if a is None:
        return b
    n = max(len(a), len(b))
    a2 = [frozenset()] * (n - len(a)) + list(a)
    b2 = [frozenset()] * (n - len(b)) + list(b)
    return tuple(x | y for x, y in zip(a2, b2))


def check(lines, name):
    blocks, order = blocks_of(lines)
    state_in = {order[0]: ()}
    work = [order[0]]
    bad = set()
    first = []
    nvm = 0
    visits = 0
    while work and visits < 20000:
        visits += 1
        lab = work.pop()
        st = list(state_in[lab])
        for t in blocks[lab][1]:
            mnem = t.split(None, 1)[0]
            rest = t.split(None, 1)[1] if " " in t else ""
            m = re.match(r"s_waitcnt\s+.*vmcnt\((\d+)\)", t)
            if m:
                keep = int(m.group(1))
                st = st[len(st) - keep:] if keep < len(st) else st
                continue
            if mnem.startswith("s_"):
                continue
            pend = set().union(*st) if st else set()
            if VMEM.match(mnem):
                nvm += 1
                if "load" in mnem:
                    dst, src = rest.split(",", 1)
                    if regs(rest) & pend:
                        bad.add(t)
                    st.append(frozenset(regs(dst)))
                else:
                    if regs(rest) & pend:
                        bad.add(t)
                    st.append(frozenset())
                st = st[-64:]
                continue
            if regs(rest) & pend:
                bad.add(t)
                if not first:
                    first.append((lab, t, [len(st) - i for i, o in enumerate(st) if o & regs(rest)]))
        out = tuple(st)
        for sname in blocks[lab][2]:
            if sname not in blocks:
                continue
            new = merge(state_in.get(sname), out)
            if new != state_in.get(sname):
                state_in[sname] = new
                work.append(sname)
    bad = sorted(bad)
    if first and "-v" in sys.argv:
        print("first hazard: block %s, %s, conflicting op(s) at depth %s" % first[0])
    print("%s: %d blocks, %d hazards%s" % (name, len(blocks), len(bad), (": " + "; ".join(bad[:6])) if bad else ""))
    return not bad


def main():
    src = open(sys.argv[1]).read()
    ok = True
    for pat in [a for a in sys.argv[2:] if a != "-v"]:
        for n in re.findall(r"^(_Z\w+):", src, re.M):
            if re.search(pat, n) and not n.startswith(".L"):
                i = src.index(n + ":")
                j = src.index(".Lfunc_end", i)
                ok &= check(src[i:j].split("\n"), n)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
