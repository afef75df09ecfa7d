#!/usr/bin/env python3
"""Dev tool: SQ counters of one rocprofv3 --pmc pass (tools/gpu_sq_pmc.sh) per
kernel class -- trace_kernel split into its binned first launch of each
propagate (the largest grid of rays, the launch after a classify) and the later
walking launches (no-op launches, < 20 us, dropped) -- as fractions of
SQ_WAVE_CYCLES (quad-cycles): parked on s_waitcnt (WAIT_ANY), issue-stalled
(WAIT_INST_ANY), issuing (ACTIVE_INST_ANY), and instructions per wave-cycle.
usage: sq_summary.py run_counter_collection.csv > summary.json"""
import csv
import json
import sys
from collections import defaultdict


def main():
    rows = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(sys.argv[1])):
        d = int(r['Dispatch_Id'])
        rows[d][r['Counter_Name']] = float(r['Counter_Value'])
        meta[d] = (r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp']))
    order = sorted(meta)
    classes = defaultdict(lambda: defaultdict(float))
    counts = defaultdict(int)
    after_classify = False
    for d in order:
        name, t0, t1 = meta[d]
        us = (t1 - t0) / 1e3
        if 'classify_kernel' in name:
            after_classify = True
        if 'trace_kernel' in name:
            if us < 20:
                continue
            cls = 'trace_first' if after_classify else 'trace_later'
            after_classify = False
        elif 'shade_kernel' in name:
            cls = 'shade'
        elif 'propagate_tail_kernel' in name:
            if us < 20:
                continue
            cls = 'tail'
        else:
            continue
        counts[cls] += 1
        classes[cls]['us'] += us
        for k, v in rows[d].items():
            classes[cls][k] += v
    out = {}
    for cls, c in classes.items():
        wc = c.get('SQ_WAVE_CYCLES', 0.0) or 1.0
        o = {'dispatches': counts[cls], 'us_per_dispatch': round(c['us'] / counts[cls], 1)}
        for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU'):
            if k in c:
                o[k.lower() + '_frac'] = round(c[k] / wc, 3)
        for k in ('SQ_INSTS_VALU', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_INSTS_SMEM'):
            if k in c:
                o[k.lower() + '_per_dispatch'] = round(c[k] / counts[cls])
                o[k.lower() + '_per_wave_quadcycle'] = round(c[k] / wc, 4)
        # the second pass's LDS counters: issue cycles and stalls as fractions of the wave
        # cycles, bank-conflict cycles against all LDS-array cycles
        for k in ('SQ_ACTIVE_INST_LDS', 'SQ_WAIT_INST_LDS'):
            if k in c:
                o[k.lower() + '_frac'] = round(c[k] / wc, 4)
        if c.get('SQ_LDS_IDX_ACTIVE'):
            o['sq_lds_bank_conflict_per_lds_cycle'] = round(c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_LDS_IDX_ACTIVE'], 4)
        for k in ('SQ_THREAD_CYCLES_VALU', 'SQ_LDS_IDX_ACTIVE', 'SQ_LDS_BANK_CONFLICT'):
            if k in c:
                o[k.lower() + '_per_dispatch'] = round(c[k] / counts[cls])
        o['wave_quadcycles_per_dispatch'] = round(wc / counts[cls])
        out[cls] = o
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
