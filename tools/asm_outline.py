"""Condensed instruction outline of one kernel in a hipcc -save-temps .s file: runs of
global loads / MFMAs / LDS reads / LDS writes / VALU, with every s_waitcnt, barrier and label.
    python tools/asm_outline.py file.s symbol_substring"""
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r'^(\S+):\s*(?:;.*)?$', s, re.M)
sym = [n for n in names if sys.argv[2] in n and not n.startswith('.')][0]
i = s.index(sym + ':')
j = s.index('.Lfunc_end', i)
out, run, cnt = [], None, 0


def kind(ins):
    if ins.startswith('v_mfma'):
        return 'MFMA'
    if ins.startswith(('global_load', 'buffer_load')):
        return 'GLOAD'
    if ins.startswith(('global_store', 'buffer_store')):
        return 'GSTORE'
    if ins.startswith('ds_read') or ins.startswith('ds_load'):
        return 'DSREAD'
    if ins.startswith('ds_write') or ins.startswith('ds_store'):
        return 'DSWRITE'
    if ins.startswith('v_'):
        return 'valu'
    if ins.startswith('s_'):
        return 'salu'
    return None


for line in s[i:j].split('\n'):
    t = line.strip()
    if not t or t.startswith(';') or t.startswith('.') and not t.startswith('.LBB'):
        continue
    if t.startswith('.LBB') or 's_waitcnt' in t or 's_barrier' in t or t.startswith('s_cbranch') or t.startswith('s_branch'):
        if run:
            out.append(f'{run}x{cnt}')
            run, cnt = None, 0
        out.append(t.split(';')[0].strip())
        continue
    k = kind(t.split()[0])
    if k is None:
        continue
    if k == run:
        cnt += 1
    else:
        if run:
            out.append(f'{run}x{cnt}')
        run, cnt = k, 1
if run:
    out.append(f'{run}x{cnt}')
print(sym)
print('\n'.join(out))
