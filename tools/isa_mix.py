"""Instruction mix of a kernel's loops in a device assembly file (hipcc --cuda-device-only -S).
python tools/isa_mix.py file.s mangled_name"""
import re, sys, collections
s = open(sys.argv[1]).read().split('\n')
name = sys.argv[2]
st = [i for i, l in enumerate(s) if l.startswith(name + ':')][0]
en = st
while not s[en].startswith('.Lfunc_end'):
    en += 1
f = s[st:en]
labels = {}
for i, l in enumerate(f):
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(f):
    m = re.search(r's_(cbranch_\w+|branch)\s+(\.LBB\S+)', l)
    if not (m and m.group(2) in labels and labels[m.group(2)] < i and i - labels[m.group(2)] > 200):
        continue
    c = collections.Counter()
    for x in f[labels[m.group(2)]:i + 1]:
        t = x.strip().split()
        if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
            continue
        op = t[0]
        k = ('v_f64' if op.startswith('v_') and 'f64' in op else 'v_dpp' if 'dpp' in op else
             'v_mov64' if op.startswith('v_mov_b64') else 'v_mov32' if op.startswith('v_mov_b32') else
             'v_cndmask' if op.startswith('v_cndmask') else 'v_other' if op.startswith('v_') else
             'vmem' if op.startswith(('global_', 'buffer_')) else 'lds' if op.startswith('ds_') else
             'waitcnt' if op.startswith('s_waitcnt') else 'branch' if op.startswith('s_cbranch') or op == 's_branch' else
             'salu' if op.startswith('s_') else op)
        c[k] += 1
    print(f'loop {labels[m.group(2)]}-{i}: {sum(c.values())} insts', dict(sorted(c.items())))
