"""Static check of the hand-counted async weight loads in a kernel's ISA: no
instruction may touch the destination registers of an inline-asm
global_load_dwordx4 before an s_waitcnt vmcnt(N) has retired it (vmcnt(N)
retires all but the N youngest vector-memory ops, counted in issue order:
loads, stores, LDS-DMA and scratch ops alike).  Linear scan: branches are
followed in program order.
usage: python tools/check_asm_loads.py file.s kernel_symbol"""
import re
import sys


def regs(tok):
    out = set()
    for m in re.finditer(r'v\[(\d+):(\d+)\]|v(\d+)\b', tok):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def main():
    path, sym = sys.argv[1], sys.argv[2]
    text = open(path).read().split('\n')
    start = next(i for i, l in enumerate(text) if l.startswith(sym + ':'))
    # the whole function (a kernel may end in several s_endpgm: warp-specialised roles)
    end = next(i for i in range(start + 1, len(text)) if text[i].startswith('.Lfunc_end'))
    pending, bad = [], 0
    for i in range(start, end):
        s = text[i].strip()
        op = s.split()[0] if s else ''
        if op.startswith(('global_load', 'buffer_load', 'global_store', 'buffer_store', 'scratch_', 'global_atomic')):
            # every VMEM op takes a vmcnt slot; only the async weight loads
            # (global_load_dwordx4 into a register quad) are tracked for hazards
            dst = regs(s.split()[1].rstrip(',')) if op == 'global_load_dwordx4' else set()
            pending.append((i, dst))
            continue
        if 's_waitcnt' in s and 'vmcnt' in s:
            n = int(re.search(r'vmcnt\((\d+)\)', s).group(1))
            pending = pending[len(pending) - n:] if n > 0 else []
            continue
        if not s or s.startswith(';') or s.startswith('.'):
            continue
        used = regs(s)
        for li, r in pending:
            if used & r:
                bad += 1
                if bad <= 10:
                    print(f"HAZARD: load at line {li + 1} -> use at line {i + 1}: {s}")
    print(f"{sym}: {bad} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
