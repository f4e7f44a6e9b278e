"""Per-kernel HBM traffic per launch from tools/pmc_bench.sh's two PMC passes.
FETCH_SIZE is doubled (gfx950 tallies 128-B requests at 64 B,
MI355X_MICROARCH.md "HBM"); WRITE_SIZE as is.  Counters are in KB.
Usage: python tools/pmc_traffic.py [gpurun_out] [cfg] > profiles/.../pmc_traffic_<cfg>.json"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, counter):
    acc = collections.defaultdict(lambda: [0.0, 0])
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] != counter:
                continue
            k = r['Kernel_Name'].split('(')[0]
            acc[k][0] += float(r['Counter_Value'])
            acc[k][1] += 1
    return acc


def main(root, cfg):
    def pdir(short, counter):     # tools/pmc_bench.sh / tools/gpu.sh pmc directory names
        d = os.path.join(root, f'pmc_{cfg}_{short}')
        return d if os.path.isdir(d) else os.path.join(root, f'pmc_{cfg}_{counter}')
    fe = load(pdir('fetch', 'FETCH_SIZE'), 'FETCH_SIZE')
    wr = load(pdir('write', 'WRITE_SIZE'), 'WRITE_SIZE')
    out = {}
    for k in sorted(set(fe) | set(wr)):
        f, nf = fe.get(k, (0.0, 0))
        w, nw = wr.get(k, (0.0, 0))
        rd = 2 * 1024 * f / nf if nf else None
        wb = 1024 * w / nw if nw else None
        out[k] = {'launches': max(nf, nw), 'read_bytes_per_launch': rd, 'write_bytes_per_launch': wb,
                  'hbm_bytes_per_launch': (rd or 0) + (wb or 0)}
    json.dump(out, sys.stdout, indent=1)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out', sys.argv[2] if len(sys.argv) > 2 else 'c3')
