"""Scan device assembly for the waitcnt anti-patterns round 6 fixed (developer
tool): a global load followed by `s_waitcnt vmcnt(0)` with no other load in
between ("isolated": one memory round trip per load -- typically a load used
only under a per-lane condition, sunk into its own branch), per kernel, with
the source lines responsible when the assembly carries line tables.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -gline-tables-only -S \\
        --cuda-device-only surreal_amd/csrc/<unit>.hip -o /tmp/unit.s
    python tools/asm_waitcnt_scan.py /tmp/unit.s [kernel-name regex]

Prints per kernel: load instructions by width, vmcnt(0) waits, isolated
loads, and (with line tables) the isolated loads' source lines.  A static
count: a hit on a path the learn never executes costs nothing."""
import collections
import re
import subprocess
import sys


def demangle(name):
    try:
        return subprocess.run(['c++filt', name], capture_output=True, text=True).stdout.strip() or name
    except OSError:
        return name


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    s = open(path).read()
    files = {int(m.group(1)): m.group(2).split('/')[-1]
             for m in re.finditer(r'\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s)}
    for m in re.finditer(r'^(_Z\w+):', s, re.M):
        name = m.group(1)
        if pat and not pat.search(name):
            continue
        end = s.find('.Lfunc_end', m.end())
        body = s[m.end():end].split('\n')
        loads = collections.Counter()
        where = collections.Counter()
        iso = 0
        loc = None
        for k, line in enumerate(body):
            lm = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', line)
            if lm:
                loc = f'{files.get(int(lm.group(1)), lm.group(1))}:{lm.group(2)}'
            mm = re.match(r'\s*((global|buffer)_load\w*)', line)
            if not mm:
                continue
            loads[mm.group(1)] += 1
            for nxt in body[k + 1:k + 16]:
                if re.match(r'\s*(global|buffer)_load', nxt):
                    break
                if 's_waitcnt vmcnt(0)' in nxt:
                    iso += 1
                    if loc:
                        where[loc] += 1
                    break
        if not loads:
            continue
        v0 = sum('vmcnt(0)' in line for line in body)
        print(f'{demangle(name)[:100]}\n    loads {dict(loads)}  vmcnt(0) {v0}  isolated {iso}')
        if where:
            print('    isolated at', ', '.join(f'{k} x{v}' for k, v in where.most_common(8)))


if __name__ == '__main__':
    main()
