"""Per-kernel table of ONE graph-replayed learn() from a rocprofv3 kernel trace
(developer tool): the learns are the runs between consecutive launches of the
first kernel of a learn; prints count / total / average microseconds per kernel
name over the median-length learn of the trace's steady state.
Usage: python tools/trace_learn.py <kernel_trace.csv> [first-kernel-substring]"""
import collections
import csv
import re
import sys


def main(path, first='zf_tmajor'):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))

    def short(n):
        return re.sub(r'^void ', '', n).split('(')[0][:60]
    st = [int(r['Start_Timestamp']) for r in rows]
    en = [int(r['End_Timestamp']) for r in rows]
    names = [short(r['Kernel_Name']) for r in rows]
    idx = [i for i, n in enumerate(names) if first in n]
    # learns: consecutive starts of the first kernel whose span is busy (graph replays)
    spans = [(a, b) for a, b in zip(idx, idx[1:]) if b - a > 20]
    good = [(a, b) for a, b in spans if (st[b] - st[a]) < 1.05 * sum(en[i] - st[i] for i in range(a, b))]
    a, b = sorted(good, key=lambda x: st[x[1]] - st[x[0]])[len(good) // 2]
    agg = collections.OrderedDict()
    for i in range(a, b):
        d = agg.setdefault(names[i], [0, 0.0])
        d[0] += 1
        d[1] += (en[i] - st[i]) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f'learn span {(st[b] - st[a]) / 1e3:.1f} us, kernels {b - a}, kernel time {tot:.1f} us')
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f'{k:60s} {v[0]:4d} {v[1]:8.1f} us  avg {v[1] / v[0]:6.2f}')


if __name__ == '__main__':
    main(*sys.argv[1:])
