#!/usr/bin/env python3
# usage: hipcc --offload-device-only -S gemm_rw.hip -o rw.s && python scripts/check_async_loads.py rw.s [kernel-regex]
"""Flag instructions that read or write a VGPR whose inline-asm load (buffer_load_dwordx4 /
global_load_dwordx4 into VGPRs) is still in flight, per kernel in a .s file.

hipcc believes an asm statement's output written when the statement issues; the data lands when
the wave's vmcnt says so.  Any use of the register before a covering ``s_waitcnt vmcnt`` -- a copy,
an address computation, an MFMA operand -- reads stale bytes.  The scan is linear over each
kernel's text (unrolled loop bodies are straight-line; LDS-DMA and stores count as VMEM ops with no
register destination), keeping after ``vmcnt(k)`` the k youngest outstanding ops.  Prints, per
kernel, the hazard count and the sequence of vmcnt waits."""
import re
import sys


def regs(tok):
    mm = re.match(r'[va]\[(\d+):(\d+)\]', tok)
    if mm:
        return {(tok[0], r) for r in range(int(mm.group(1)), int(mm.group(2)) + 1)}
    mm = re.match(r'([va])(\d+)$', tok)
    return {(mm.group(1), int(mm.group(2)))} if mm else set()


def scan(body):
    lines = [l.strip() for l in body.split('\n')]
    pending, bad, vm, where = [], 0, [], []
    for n, l in enumerate(lines):
        if not l or l.startswith(';') or l.startswith('.') or l.endswith(':'):
            continue
        op = l.split()[0]
        toks = l.replace(',', ' ').split()[1:]
        if op.startswith(('buffer_load', 'global_load')) and 'lds' not in toks and '_lds' not in op:
            pending.append(regs(toks[0]))
            continue
        if op.startswith(('buffer_', 'global_', 'flat_', 'scratch_')):
            pending.append(set())
            continue
        if op == 's_waitcnt' and 'vmcnt' in l:
            k = int(re.search(r'vmcnt\((\d+)\)', l).group(1))
            vm.append(k)
            pending = pending[-k:] if k else []
            continue
        if op.startswith('s_'):
            continue
        used = set()
        for t in toks:
            used |= regs(t)
        for d in pending:
            if used & d:
                bad += 1
                if len(where) < 3:
                    where.append(f"{n}: {l}")
                break
    return bad, vm, where


def main(argv):
    s = open(argv[1]).read()
    pat = argv[2] if len(argv) > 2 else r'_ZN4dllm14gemm_rw_kernel\w+'
    for m in re.finditer(rf'^({pat}):', s, re.M):
        name = m.group(1)
        body = s[m.end(): s.index('.Lfunc_end', m.end())]
        bad, vm, where = scan(body)
        print(name[:56], 'hazards', bad, 'vmcnt', vm[:8], '...', vm[-2:])
        for w in where:
            print('   ', w)


if __name__ == '__main__':
    main(sys.argv)
