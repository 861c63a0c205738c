"""Static check of the hand-counted async weight loads in a kernel's ISA: no
instruction may touch the destination registers of an inline-asm
global_load_dwordx4 before an s_waitcnt vmcnt(N) has retired it (vmcnt(N)
retires all but the N youngest vector-memory ops, counted in issue order:
loads, stores, LDS-DMA and scratch ops alike).

Control flow is followed, not just program order: the function is split into
basic blocks (labels, branches, s_endpgm), and the queue of vector-memory ops
still in flight is propagated along every edge -- including loop back-edges --
to a fixpoint.  A block's entry state is the set of queues any path can reach
it with, so a load issued at a loop's tail and used at its head on the next
trip (v5 issues weights two groups ahead, across chunk and tile iterations) is
seen, whatever the entry path's waits say.
usage: python tools/check_asm_loads.py file.s kernel_symbol"""
import re
import sys

VMCNT_MAX = 63          # the hardware counter's range: older ops are retired by then anyway
MAX_STATES = 4096       # per block: a guard against a pathological state explosion


def regs(tok):
    out = set()
    for m in re.finditer(r'v\[(\d+):(\d+)\]|v(\d+)\b', tok):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def is_vmem(op):
    return op.startswith(('global_load', 'buffer_load', 'global_store', 'buffer_store', 'scratch_',
                          'global_atomic', 'buffer_atomic'))


def parse(lines):
    """-> (instrs, labels): instrs = [(line_no, text, op)], labels = {label: index of next instr}."""
    instrs, labels = [], {}
    for no, raw in lines:
        s = raw.split(';')[0].strip()
        if not s:
            continue
        if s.endswith(':'):
            labels[s[:-1]] = len(instrs)
            continue
        if s.startswith('.'):
            continue
        instrs.append((no, s, s.split()[0]))
    return instrs, labels


def blocks_of(instrs, labels):
    """Basic blocks as [start, end) instruction ranges and their successor block starts."""
    starts = {0} | {i for i in labels.values() if i < len(instrs)}
    for i, (_, s, op) in enumerate(instrs):
        if op.startswith(('s_branch', 's_cbranch', 's_endpgm', 's_setpc', 's_trap')) and i + 1 < len(instrs):
            starts.add(i + 1)
    order = sorted(starts)
    succ = {}
    for k, b in enumerate(order):
        e = order[k + 1] if k + 1 < len(order) else len(instrs)
        _, s, op = instrs[e - 1]
        nxt = []
        if op.startswith('s_branch'):
            nxt = [labels[s.split()[1]]]
        elif op.startswith('s_cbranch'):
            nxt = [labels[s.split()[1]]] + ([e] if e < len(instrs) else [])
        elif op.startswith(('s_endpgm', 's_setpc', 's_trap')):
            nxt = []
        elif e < len(instrs):
            nxt = [e]
        succ[b] = (e, [n for n in nxt if n < len(instrs)])
    return succ


UNTRACKED = (0, frozenset())


def step(queue, no, s, op):
    """Queue after one instruction (queue: tuple of (load line, frozenset(dst regs)), oldest first)."""
    if is_vmem(op):
        # every VMEM op takes a vmcnt slot; only the async weight loads
        # (global_load_dwordx4 into a register quad) are tracked for hazards
        # (untracked ops are interchangeable: only their count matters)
        parts = s.split()
        if op == 'global_load_dwordx4' and len(parts) > 1:
            q = queue + ((no, frozenset(regs(parts[1].rstrip(',')))),)
        else:
            q = queue + (UNTRACKED,)
        return q[-VMCNT_MAX:]
    if op == 's_waitcnt' and 'vmcnt' in s:
        n = int(re.search(r'vmcnt\((\d+)\)', s).group(1))
        return queue[len(queue) - n:] if 0 < n < len(queue) else (queue if n >= len(queue) else ())
    return queue


def check(lines, verbose=True):
    """Number of hazards (instruction uses a register of an unretired tracked load) over all paths."""
    instrs, labels = parse(lines)
    if not instrs:
        return 0
    succ = blocks_of(instrs, labels)
    entry = {b: set() for b in succ}
    entry[0].add(())
    work = [0]
    hazards = {}
    while work:
        b = work.pop()
        e, nxt = succ[b]
        outs = set()
        for q0 in entry[b]:
            q = q0
            for i in range(b, e):
                no, s, op = instrs[i]
                used = regs(s) if not is_vmem(op) or op != 'global_load_dwordx4' else regs(s.split(None, 1)[1]) - \
                    regs(s.split()[1].rstrip(','))
                if used:
                    for (ls, r) in q:
                        if r and used & r:
                            hazards.setdefault((no, ls), s)
                q = step(q, no, s, op)
            outs.add(q)
        for n in nxt:
            before = len(entry[n])
            entry[n] |= outs
            if len(entry[n]) > MAX_STATES:
                raise RuntimeError(f"state explosion at block {n}")
            if len(entry[n]) != before and n not in work:
                work.append(n)
    if verbose:
        for k, ((no, ls), s) in enumerate(sorted(hazards.items())):
            if k >= 10:
                break
            print(f"HAZARD: load at line {ls} still in flight at line {no}: {s}")
    return len(hazards)


def function_lines(text, sym):
    lines = text.split('\n')
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ':'))
    # the whole function (a kernel may end in several s_endpgm: warp-specialised roles)
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith('.Lfunc_end'))
    return [(i + 1, lines[i]) for i in range(start + 1, end)]


def main():
    path, sym = sys.argv[1], sys.argv[2]
    bad = check(function_lines(open(path).read(), sym))
    print(f"{sym}: {bad} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
