"""Rough VGPR liveness of one kernel in a gfx950 .s file (no GPU needed): CFG from labels and
branches, backward dataflow, the peak live count and what is live there.
usage: python3 scripts/vlive.py file.s kernel_symbol [top]"""
import re, sys, collections
src = open(sys.argv[1]).read().split('\n')
sym = sys.argv[2]
i0 = next(i for i, l in enumerate(src) if l.startswith(sym + ':'))
i1 = next(i for i in range(i0 + 1, len(src)) if src[i].startswith('.Lfunc_end'))
RE = re.compile(r'\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]')
def regs(tok):
    out = []
    for m in RE.finditer(tok):
        if m.group(1): out.append(f'{m.group(1)}{m.group(2)}')
        else: out += [f'{m.group(3)}{k}' for k in range(int(m.group(4)), int(m.group(5)) + 1)]
    return out
NODEF = ('buffer_store', 'global_store', 'ds_write', 'global_atomic_add ', 's_', 'v_cmp_', 'v_readlane', 'v_readfirstlane',
         'scratch_store', 'buffer_atomic', 'ds_write2')
blocks = []; cur = {'label': None, 'ins': []}
for ln in src[i0 + 1:i1]:
    s = ln.split(';')[0].strip()
    if not s or (s.startswith('.') and not re.match(r'^\.LBB\d+_\d+:', s)): continue
    m = re.match(r'^(\.LBB\d+_\d+):', s)
    if m:
        blocks.append(cur); cur = {'label': m.group(1), 'ins': []}; continue
    cur['ins'].append(s)
    op = s.split()[0]
    if op.startswith('s_branch') or op.startswith('s_cbranch') or op == 's_endpgm':
        blocks.append(cur); cur = {'label': None, 'ins': []}
blocks.append(cur)
blocks = [b for b in blocks if b['ins'] or b['label']]
lab = {b['label']: k for k, b in enumerate(blocks) if b['label']}
def parse(s):
    op = s.split()[0]
    rest = s[len(op):]
    ops = [o.strip() for o in rest.split(',')]
    if op.startswith(NODEF) or op.startswith('v_cmpx'):
        if op.startswith('v_cmp_') and op.endswith('_e32'): return set(), set(regs(rest))
        return set(), set(regs(rest))
    d = set(regs(ops[0])) if ops and ops[0] else set()
    u = set(regs(','.join(ops[1:])))
    if op.startswith('v_writelane') or 'dpp' in op and 'bound_ctrl' not in s: u |= d
    if op.startswith('v_cndmask') or op.startswith('v_div_fmas'): pass
    return d, u
for b in blocks:
    b['pi'] = [parse(s) for s in b['ins']]
succ = []
for k, b in enumerate(blocks):
    ss = []
    last = b['ins'][-1] if b['ins'] else ''
    op = last.split()[0] if last else ''
    if op.startswith('s_branch') or op.startswith('s_cbranch'):
        t = last.split()[1]
        if t in lab: ss.append(lab[t])
    if not (op.startswith('s_branch') or op == 's_endpgm') and k + 1 < len(blocks): ss.append(k + 1)
    succ.append(ss)
livein = [set() for _ in blocks]
changed = True
while changed:
    changed = False
    for k in range(len(blocks) - 1, -1, -1):
        live = set().union(*[livein[j] for j in succ[k]]) if succ[k] else set()
        for d, u in reversed(blocks[k]['pi']):
            live = (live - d) | u
        if live != livein[k]: livein[k] = live; changed = True
peak = (0, None, None)
hist = collections.Counter()
for k, b in enumerate(blocks):
    live = set().union(*[livein[j] for j in succ[k]]) if succ[k] else set()
    for idx in range(len(b['ins']) - 1, -1, -1):
        d, u = b['pi'][idx]
        n = len([r for r in live if r[0] == 'v'])
        if n > peak[0]: peak = (n, k, idx)
        live = (live - d) | u
top = int(sys.argv[3]) if len(sys.argv) > 3 else 0
print('blocks', len(blocks), 'peak live VGPRs', peak[0], 'at block', peak[1], blocks[peak[1]]['label'], 'ins', peak[2])
print('live-in per block (VGPRs):', [(k, blocks[k]['label'], len([r for r in livein[k] if r[0]=='v']), len(blocks[k]['ins'])) for k in range(len(blocks)) if len(blocks[k]['ins']) > 40][:top or 60])
if len(sys.argv) > 4:
    for k in range(int(sys.argv[4]), int(sys.argv[5]) + 1):
        b = blocks[k]
        live = set().union(*[livein[j] for j in succ[k]]) if succ[k] else set()
        cnt = []
        for idx in range(len(b['ins']) - 1, -1, -1):
            d, u = b['pi'][idx]
            cnt.append(len([r for r in live if r[0] == 'v']))
            live = (live - d) | u
        cnt.reverse()
        print(f'== block {k} {b["label"]} succ {succ[k]} livein {len([r for r in livein[k] if r[0]=="v"])}')
        for s, c in zip(b['ins'], cnt): print(f'  {c:4d}  {s}')
