"""Per-kernel durations and the idle gaps in front of them, from a rocprofv3
--kernel-trace CSV (eager learns: graph replays are inflated under the tracer).

    python tools/trace_gaps.py <dir with *kernel_trace.csv> [--last N]

Prints, per kernel name (template arguments cut), launches, mean duration and
mean gap from the previous kernel's end to this kernel's start (same queue),
over the dispatches of the last N learn() calls (a learn() ends with its
rnn_final_kernel launch)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split('(')[0]
    for p in ('void ', 'smi::'):
        n = n.replace(p, '')
    return n[:60]


def main():
    d = sys.argv[1]
    last = int(sys.argv[sys.argv.index('--last') + 1]) if '--last' in sys.argv else 3
    fs = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)
    if not fs:
        raise SystemExit('no kernel_trace.csv under ' + d)
    rows = []
    for f in fs:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if 'rnn_final_kernel' in r[2]]
    if len(ends) > last:
        rows = rows[ends[-last - 1] + 1:ends[-1] + 1]
    dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
    prev_end = None
    for s, e, n in rows:
        k = short(n)
        dur[k] += (e - s) / 1e3
        if prev_end is not None:
            gap[k] += max(0, s - prev_end) / 1e3
        cnt[k] += 1
        prev_end = e
    span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0.0
    tot_d = sum(dur.values())
    tot_g = sum(gap.values())
    n_learn = max(1, last)
    print(f'{len(rows)} dispatches over {n_learn} learn() calls: span {span / n_learn:.1f} us per learn, '
          f'kernels {tot_d / n_learn:.1f} us, gaps {tot_g / n_learn:.1f} us')
    for k in sorted(dur, key=lambda x: -dur[x] - gap[x]):
        c = cnt[k]
        print(f'  {k:60s} x{c / n_learn:6.1f}/learn  dur {dur[k] / c:7.2f} us  gap {gap[k] / c:6.2f} us  '
              f'total {(dur[k] + gap[k]) / n_learn:8.1f} us/learn')


if __name__ == '__main__':
    main()
