"""Count the instructions of one kernel in a hipcc -S listing: python tools/isa_count.py file.s substring"""
import collections
import sys

s = open(sys.argv[1]).read()
names = [l.split(':')[0] for l in s.split('\n') if sys.argv[2] in l and l.endswith(':') is False and l.startswith('_Z')
         and ':' in l]
name = names[0]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
c = collections.Counter()
for l in s[i:j].split('\n'):
    l = l.strip()
    if not l or l.startswith(('.', ';')) or l.endswith(':'):
        continue
    c[l.split()[0]] += 1
print(name)
print('valu', sum(v for k, v in c.items() if k.startswith('v_')), 'total', sum(c.values()))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30):
    print(' ', k, v)
