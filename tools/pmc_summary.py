"""Per-kernel PMC summary of rocprofv3 --pmc runs: every counter averaged over
the dispatches of each (kernel, grid size), plus the derived ratios the
kernel work in DESIGN.md quotes (MFMA busy share of wave cycles, wait shares).
Usage: python tools/pmc_summary.py DIR [DIR ...]  (each DIR: one or more
--pmc passes of the same command, *counter_collection.csv anywhere below)"""
import collections
import csv
import glob
import json
import os
import sys


def load(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            for r in csv.DictReader(open(f)):
                k = (r['Kernel_Name'].split('(')[0].split('<')[0].strip(), int(r.get('Grid_Size', 0) or 0))
                acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
    return acc


def main(dirs):
    acc = load(dirs)
    out = {}
    for (name, grid), cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {'dispatches': max(len(v) for v in cs.values())}
        d.update({c: round(v, 1) for c, v in m.items()})
        wc = m.get('SQ_WAVE_CYCLES')
        if wc:
            for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY'):
                if c in m:
                    d[c + '/WAVE_CYCLES'] = round(m[c] / wc, 3)
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in m and 'SQ_BUSY_CYCLES' in m and m['SQ_BUSY_CYCLES']:
            d['MFMA_BUSY/SQ_BUSY'] = round(m['SQ_VALU_MFMA_BUSY_CYCLES'] / m['SQ_BUSY_CYCLES'], 3)
        if 'TCC_HIT_sum' in m and 'TCC_MISS_sum' in m and m['TCC_HIT_sum'] + m['TCC_MISS_sum']:
            d['L2_hit'] = round(m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']), 3)
        out[f'{name}@{grid}'] = d
    json.dump(out, sys.stdout, indent=1)


if __name__ == '__main__':
    main(sys.argv[1:])
