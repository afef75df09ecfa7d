#!/usr/bin/env python
"""Summarise a tools/gather_calib run (tools/gpu_r02_diag.sh): per kernel, the
bytes it requested, the 64-B sectors and 128-B lines they span, rocprofv3's
FETCH_SIZE and its average duration, and the ratios that calibrate FETCH_SIZE
for the BVH walk's gathers.  usage: tools/gather_calib.py DIR > out.json"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    calib = json.load(open(os.path.join(d, 'calib.json')))
    fetch = {}
    for f in glob.glob(os.path.join(d, 'calib_fetch', '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == 'FETCH_SIZE':
                k = r['Kernel_Name'].split('(')[0].replace('void ', '')
                fetch[k] = fetch.get(k, 0.0) + float(r['Counter_Value']) * 1024.0
    dur = {}
    for f in glob.glob(os.path.join(d, 'calib_trace', '**', '*kernel_stats.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r['Name'].split('(')[0].replace('void ', '')] = float(r['AverageNs'])
    out = []
    for c in calib:
        k = c['kernel']
        fb = fetch.get(k)
        row = dict(c, fetch_size_bytes=fb, avg_ns=dur.get(k))
        if fb:
            row['fetch_over_lines128'] = fb / c['lines128']
            row['fetch_x2_over_lines128'] = 2 * fb / c['lines128']
            row['fetch_x2_over_requested'] = 2 * fb / c['bytes']
        if dur.get(k):
            row['lines128_GBps'] = c['lines128'] / dur[k]
        out.append(row)
    json.dump({'source': d, 'kernels': out,
               'finding': 'FETCH_SIZE = 64 B per 128-B line request for every access shape (coalesced stream and '
                          'random 16/48/64/96/128-B gathers alike): x2 gives the bytes the lines move'},
              sys.stdout, indent=1)


if __name__ == '__main__':
    main()
