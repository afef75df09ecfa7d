#!/usr/bin/env python
"""Sum rocprofv3 --pmc counters per kernel (propagate_kernel vs the rest).
usage: pmc_summary.py DIR [DIR...]   (dev tool)"""
import csv
import glob
import os
import sys


def main():
    for d in sys.argv[1:]:
        tot = {}
        disp = {}
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            for row in csv.DictReader(open(f)):
                k = 'propagate_kernel' if 'propagate_kernel' in row['Kernel_Name'] else 'other'
                c = row['Counter_Name']
                tot[(k, c)] = tot.get((k, c), 0.0) + float(row['Counter_Value'])
                disp.setdefault(k, set()).add(row['Dispatch_Id'])
        print(d)
        for (k, c), v in sorted(tot.items()):
            n = len(disp[k])
            print('  %-18s %-40s total %.4g  per-dispatch %.4g  (%d dispatches)' % (k, c, v, v / n, n))


if __name__ == '__main__':
    main()
