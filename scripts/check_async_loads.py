#!/usr/bin/env python3
# usage: hipcc ... -S gemm_gu.hip -o gu.s && python scripts/check_async_loads.py gu.s
"""Flag non-MFMA instructions that read or write a VGPR with an asm global_load still in flight
(no vmcnt wait since), per kernel in a .s file."""
import re, sys
s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_ZN4dllm15gemm_gua_kernel\w+):', s, re.M):
    name = m.group(1); i = m.end(); j = s.index('.Lfunc_end', i)
    lines = [l.strip() for l in s[i:j].split('\n')]
    def regs(tok):
        mm = re.match(r'v\[(\d+):(\d+)\]', tok)
        if mm: return set(range(int(mm.group(1)), int(mm.group(2)) + 1))
        mm = re.match(r'v(\d+)$', tok)
        return {int(mm.group(1))} if mm else set()
    pending = []; bad = 0; vm = []
    for n, l in enumerate(lines):
        if l.startswith('global_load_dwordx4'):
            parts = l.replace(',', ' ').split(); pending.append(regs(parts[1])); continue
        if l.startswith('global_load_lds') or l.startswith('buffer_load') or l.startswith('global_store') or l.startswith('global_load'):
            pending.append(set())
        if l.startswith('s_waitcnt') and 'vmcnt' in l:
            k = int(re.search(r'vmcnt\((\d+)\)', l).group(1)); vm.append(k)
            # conservatively keep the youngest k entries (other VMEM ops counted too -> over-keep)
            pending = pending[-k:] if k else []
            continue
        if not l or l.startswith(';') or l.startswith('.') or l.startswith('v_mfma') or l.startswith('s_'): continue
        used = set()
        for t in l.replace(',', ' ').split()[1:]: used |= regs(t)
        for d in pending:
            if used & d:
                bad += 1
                if bad < 3: print('   ', n, l)
    print(name[:48], 'hazards', bad, 'vmcnt', vm[:8], '...', vm[-2:])
