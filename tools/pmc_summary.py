#!/usr/bin/env python
"""Sum rocprofv3 --pmc counters per kernel (grouped by kernel name with its
template arguments).  usage: pmc_summary.py DIR [DIR...]   (dev tool)"""
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r'(propagate_(?:step_)?kernel<[^>]*>)', name)
    return m.group(1) if m else name.split('(')[0][-60:]


def main():
    for d in sys.argv[1:]:
        tot = {}
        disp = {}
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            for row in csv.DictReader(open(f)):
                k = short(row['Kernel_Name'])
                c = row['Counter_Name']
                tot[(k, c)] = tot.get((k, c), 0.0) + float(row['Counter_Value'])
                disp.setdefault(k, set()).add(row['Dispatch_Id'])
        print(d)
        for (k, c), v in sorted(tot.items()):
            if 'propagate' not in k:
                continue
            n = len(disp[k])
            print('  %-42s %-28s total %.4g  per-dispatch %.4g  (%d dispatches)' % (k, c, v, v / n, n))


if __name__ == '__main__':
    main()
