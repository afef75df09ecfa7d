#!/usr/bin/env python3
"""Per-kernel time of a rocprofv3 kernel trace (CSV), per propagate.

usage: tools/rocprof_breakdown.py kernel_trace.csv[.gz] [propagates]
The per-slot tail launches on the tail stream that find their slot not in
tail mode exit at once, but a launch queued behind a persistent trace grid
shows the whole wait as its duration; they are reported apart ("tail (slot
not in tail mode)": launches whose grid ran no photon, told from the real
tails by their duration, < 50 us once dispatched -- their start is taken as
the end of the trace launch running when they were queued)."""
import csv
import gzip
import json
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(gzip.open(path, 'rt') if path.endswith('.gz') else open(path)))
    S = lambda r: int(r['Start_Timestamp'])   # noqa: E731
    E = lambda r: int(r['End_Timestamp'])     # noqa: E731
    nprop = int(sys.argv[2]) if len(sys.argv) > 2 else max(1, sum('init_queue' in r['Kernel_Name'] for r in rows))
    rows.sort(key=S)
    traces = [(S(r), E(r)) for r in rows if 'trace_kernel' in r['Kernel_Name']]
    tot = defaultdict(float)
    calls = defaultdict(int)
    for r in rows:
        name = r['Kernel_Name'].split('(')[0].replace('void ', '')
        if name.startswith('rocprim'):
            name = 'rocprim radix sort'
        d = (E(r) - S(r)) / 1e6
        if 'propagate_tail_kernel' in name:
            # time after the overlapping trace launch (if any) ended: what the tail itself took
            s = S(r)
            for a, b in traces:
                if a <= s < b:
                    s = b
                    break
            own = max(0.0, (E(r) - s) / 1e6)
            name = 'propagate_tail_kernel' if own >= 0.05 else 'propagate_tail_kernel (slot not in tail mode)'
            d = own
        tot[name] += d
        calls[name] += 1
    total = sum(tot.values())
    out = {'propagates': nprop, 'kernel_ms_per_propagate': round(total / nprop, 3), 'kernels': []}
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        if v / nprop < 0.005:
            continue
        out['kernels'].append({'name': k, 'ms_per_propagate': round(v / nprop, 3), 'calls': calls[k],
                               'share': round(v / total, 4)})
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
