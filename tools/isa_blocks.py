"""Basic blocks of one kernel in a device assembly listing, with their
instruction counts by class (VALU, SALU, global/buffer, LDS) and branch
targets: the loop bodies of a hot kernel and what they issue.
  hipcc <flags> --cuda-device-only -S -o api.s mantis_amd/csrc/api.hip
  python tools/isa_blocks.py api.s <first line> <last line of the function>"""
import re,sys,collections
lines=open(sys.argv[1]).read().split('\n')
a,b=int(sys.argv[2]),int(sys.argv[3])
blocks=[];cur=None
for i in range(a,b):
    l=lines[i]
    m=re.match(r'^(\.LBB\d+_\d+|\S+):',l)
    if m: cur=[m.group(1),i+1,[]];blocks.append(cur);continue
    s=l.strip()
    if not s or s.startswith(';') or s.startswith('.'): continue
    if cur is None: cur=['entry',i+1,[]];blocks.append(cur)
    cur[2].append(s)
for name,ln,ins in blocks:
    c=collections.Counter()
    br=[]
    for s in ins:
        op=s.split()[0]
        if op.startswith('v_'): c['v']+=1
        elif op.startswith('s_'): c['s']+=1
        elif op.startswith('global_') or op.startswith('buffer_'): c['g']+=1
        elif op.startswith('ds_'): c['ds']+=1
        if op.startswith('s_cbranch') or op=='s_branch': br.append(s.split()[1])
    print(f"{name:16s} L{ln:6d} n={len(ins):4d} v={c['v']:4d} s={c['s']:4d} g={c['g']:3d} ds={c['ds']:3d} br={br}")
