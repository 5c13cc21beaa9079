"""Static instruction mix between consecutive s_memtime stamps of wbc_update_solve_kernel in a
WBC_ISTAMPS listing (hipcc -S -gline-tables-only -DWBC_ISTAMPS): each segment is labelled with the
source line of the stamp that opens it.  Usage: python tools/ust_segments.py listing.s [line ...]"""
import re
import sys

path = sys.argv[1]
want = {int(a) for a in sys.argv[2:]}
s = open(path).read().split('\n')
st = [i for i, l in enumerate(s) if l.startswith('_ZN3wbc23wbc_update_solve_kernelENS_10KernelArgsE:')][0]
en = [i for i, l in enumerate(s[st:]) if l.startswith('.Lfunc_end')][0] + st
new = lambda: dict(valu=0, ds=0, wait=0, acc=0, dpp=0)
seg, cur, loc, lab = [], new(), None, None
for l in s[st:en]:
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
    if m:
        loc = int(m.group(2))
        continue
    t = l.strip()
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    if t.startswith('s_memtime'):
        seg.append((lab, cur))
        cur, lab = new(), loc
        continue
    op = t.split()[0]
    if op.startswith('v_'):
        cur['valu'] += 1
        cur['dpp'] += ('dpp' in t or 'row_' in t)
        cur['acc'] += ('accvgpr' in op)
    elif op.startswith('ds_'):
        cur['ds'] += 1
    elif op.startswith('s_waitcnt'):
        cur['wait'] += 1
seg.append((lab, cur))
for i, (lab, c) in enumerate(seg):
    if not want or lab in want:
        print(i, lab, c)
