"""Kernels whose vector loads go out one at a time (lab tool).

    hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -Iinclude -x hip --cuda-device-only -S amg_amd/csrc/X.hip -o X.s
    python tools/serial_scan.py X.s ...

For each kernel: global loads, and how many of them are followed by an `s_waitcnt vmcnt(0)` before
the next global load is issued -- i.e. the wave waits for that load (and every older one) before it
can put another in flight.  A gather loop compiled with the multiply (or the store) under the
load's condition shows up here as one wait per gather.
"""
import re
import sys

for path in sys.argv[1:]:
    lines = open(path).read().splitlines()
    name, stats, pending = None, {}, False
    for l in lines:
        m = re.match(r'^(_Z\w+):', l)
        if m:
            name, pending = m.group(1), False
            stats[name] = [0, 0]
            continue
        if not name:
            continue
        t = l.strip()
        if t.startswith('global_load') or t.startswith('buffer_load'):
            stats[name][0] += 1
            pending = True
        elif pending and 's_waitcnt' in t and 'vmcnt(0)' in t:
            stats[name][1] += 1
            pending = False
        elif t.startswith('s_endpgm'):
            pending = False
    for k, (a, b) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        if b >= 6:
            print(f"{b:3d}/{a:3d}  {k[:120]}")
