#!/usr/bin/env python3
"""Tabulate scripts/tune_tile.py logs: us per turn (with counts) per size, tile T (rows) x depth K."""
import json
import sys

for f in sys.argv[1:]:
    txt = open(f).read()
    j = json.loads(txt[txt.index('{'):txt.index('\nbest')] if '\nbest' in txt else txt[txt.index('{'):])
    d = j['us_per_turn_with_counts']
    for s in sorted({int(k.split('/')[0]) for k in d}):
        print('size', s)
        Ts = sorted({k.split('/')[1] for k in d if k.startswith(f'{s}/')})
        Ks = sorted({int(k.split('/')[2][1:]) for k in d if k.startswith(f'{s}/')})
        print('        ' + ''.join(f'   k{k:<7d}' for k in Ks))
        for T in Ts:
            print(f'{T:7s} ' + ''.join(f"{d[f'{s}/{T}/k{k}']['us_per_turn']:7.3f}{d[f'{s}/{T}/k{k}']['kind'][:2]:>3s} "
                                       for k in Ks))
