"""Static instruction counts of one kernel in a `hipcc -S -gline-tables-only` listing, by source
line range of wbc_kernel.hip (diagnostic: where the instructions, AGPR moves, LDS ops and waits sit).
Usage: python tools/isa_lines.py listing.s kernel_symbol A-B [C-D ...]"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split('\n')
st = [i for i, l in enumerate(lines) if l.startswith(sym + ':')][0]
en = [i for i, l in enumerate(lines[st:]) if l.startswith('.Lfunc_end')][0] + st
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[int(m.group(1))] = (m.group(3) or m.group(2))
cur = None
rows = []
for l in lines[st:en]:
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
    if m:
        cur = (int(m.group(1)), int(m.group(2)))
        continue
    t = l.strip()
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    rows.append((cur, t))
def stats(a, b):
    s = dict(instr=0, valu=0, acc=0, ds=0, wait=0, dpp=0)
    for (cur, t) in rows:
        if cur is None or 'wbc_kernel' not in files.get(cur[0], '') or not (a <= cur[1] <= b):
            continue
        s['instr'] += 1
        if t.startswith('v_'):
            s['valu'] += 1
        if t.startswith('v_accvgpr'):
            s['acc'] += 1
        if t.startswith('ds_'):
            s['ds'] += 1
        if t.startswith('s_waitcnt'):
            s['wait'] += 1
        if 'dpp' in t or 'row_' in t or 'quad_perm' in t:
            s['dpp'] += 1
    return s
print("total", len(rows))
for r in sys.argv[3:]:
    a, b = map(int, r.split('-'))
    print(r, stats(a, b))
