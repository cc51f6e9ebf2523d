"""Instruction mix of the backward-branch loops of one kernel in a device .s file:
python tools/loop_mix.py file.s kernel_substring"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
names = [m.group(1) for m in re.finditer(r'^(\S+):(?:\s*;.*)?$', s, re.M) if key in m.group(1) and not m.group(1).startswith('.')]
for name in names:
    body = s[s.index(name + ':'):]
    body = body[:body.index('.Lfunc_end')]
    lines = body.split('\n')
    labels = {l.strip().split(':')[0]: i for i, l in enumerate(lines) if re.match(r'^\.LBB\S+:', l.strip())}
    for i, l in enumerate(lines):
        m = re.match(r'\s*s_cbranch_\w+\s+(\.LBB\S+)', l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            a = labels[m.group(1)]
            c = collections.Counter()
            for x in lines[a:i]:
                t = x.strip().split()
                if not t or t[0].startswith(('.', ';')):
                    continue
                op = t[0]
                if op.startswith('v_mfma'):
                    c['MFMA'] += 1
                elif op.startswith('v_'):
                    c['VALU'] += 1
                    c[op] += 1
                elif op.startswith('ds_'):
                    c['LDS'] += 1
                elif op.startswith(('global_', 'buffer_')):
                    c['VMEM'] += 1
                elif op.startswith('s_'):
                    c['SALU/branch'] += 1
            print(name[:60], m.group(1), dict(c.most_common(24)))
