import json, sys
lines = open(sys.argv[1]).read().splitlines()
d = json.loads([l for l in lines if l.startswith('{')][0])
vs = sorted(set(k.split('_')[0] for k in d))
for v in vs:
    ks = sorted(set(int(k.split('_')[1][1:]) for k in d if k.startswith(v)))
    bs = sorted(set(int(k.split('_b')[1]) for k in d if k.startswith(v)))
    print(v, 'band', bs)
    for k in ks:
        print('  k%-3d' % k, [d.get(f'{v}_k{k}_b{b}') for b in bs])
print([l for l in lines if l.startswith('best')])
