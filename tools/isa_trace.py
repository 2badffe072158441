"""Compressed instruction-class trace of one kernel in a hipcc --save-temps .s:
M = MFMA, L = global load, S = global store, W(..) = s_waitcnt, X = scratch.
    python tools/isa_trace.py file.s mangled_prefix"""
import sys

s = open(sys.argv[1]).read()
start = s.index(sys.argv[2] + ':')
end = s.index('.Lfunc_end', start)
seq = []
for l in s[start:end].split('\n'):
    t = l.strip().split(' ')[0]
    if not t or t.startswith(';'):
        continue
    if t.startswith('.LBB'):
        seq.append(t)
        continue
    if t.startswith('.'):
        continue
    if 'mfma' in t:
        c = 'M'
    elif t.startswith('global_load'):
        c = 'L'
    elif t.startswith('s_waitcnt'):
        c = 'W(' + l.strip().split(' ', 1)[1] + ')'
    elif t.startswith('s_cbranch') or t.startswith('s_branch'):
        c = 'B:' + l.strip().split(' ', 1)[1]
    elif t.startswith('global_store'):
        c = 'S'
    elif t.startswith('scratch') or t.startswith('buffer_'):
        c = 'X'
    elif t.startswith('v_accvgpr'):
        c = 'a'
    else:
        c = '.'
    seq.append(c)
out, prev, n = [], None, 0
for c in seq + [None]:
    if c == prev:
        n += 1
        continue
    if prev is not None:
        out.append(f'{prev}x{n}' if n > 1 else prev)
    prev, n = c, 1
print(' '.join(out))
