#!/usr/bin/env python
"""Summarise the FETCH_SIZE / WRITE_SIZE passes of tools/rocprof_bench.sh into
HBM bytes per propagate-kernel launch (MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are rocprofv3 derived counters in KiB; on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced reads, so it is doubled here -- an upper-bound
correction for the narrower gathers of the BVH walk, whose calibration is
unknown).  Prints one JSON object."""
import csv
import re
import glob
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get('Counter_Name') != counter:
                    continue
                name = row.get('Kernel_Name', '')
                key = (row.get('Dispatch_Id'), name)
                vals[key] = vals.get(key, 0.0) + float(row['Counter_Value'])
    out = {}
    for (_, name), v in vals.items():
        out.setdefault(kernel_class(name), []).append(v)
    return out


def kernel_class(name):
    """Kernels of the propagate path by role (the counting variant, run untimed
    by bench.py, is kept apart)."""
    if ', true>' in name:
        return 'counting_variant'
    if 'trace_kernel' in name:
        return 'chr::trace_kernel'
    if re.search(r'propagate_step_kernel<[^>]*9000', name):
        return 'chr::propagate_step_kernel (shade)'
    if re.search(r'propagate_(step_)?kernel<', name):
        return 'chr::propagate_step_kernel (fused walk + shade)'
    return name.split('(')[0]


def main():
    d = sys.argv[1]
    fetch = per_kernel(os.path.join(d, 'fetch'), 'FETCH_SIZE')
    write = per_kernel(os.path.join(d, 'write'), 'WRITE_SIZE')
    k = 'chr::trace_kernel'     # the dominant kernel (bench.py roofline)
    res = {'kernel': k}
    # device-driven steps launch trace_kernel in every step slot; in the tail's
    # and the idle slots it reads its mode word and exits (a few KiB): the
    # per-launch figures are over the launches that walked rays (>= 64 KiB;
    # a one-step launch holds >= 65,536 rays and writes 8 B of hit per ray)
    for dct in (fetch, write):
        if k in dct:
            dct[k + ' (exited)'] = [v for v in dct[k] if v < 64.0]
            dct[k] = [v for v in dct[k] if v >= 64.0]
    if k in fetch:
        f = fetch[k]
        res['launches_fetch_pass'] = len(f)
        res['exited_launches_fetch_pass'] = len(fetch.get(k + ' (exited)', []))
        res['fetch_kib_per_launch_raw'] = sum(f) / len(f)
        res['read_bytes_per_launch'] = 2.0 * 1024.0 * sum(f) / len(f)
    if k in write:
        w = write[k]
        res['launches_write_pass'] = len(w)
        res['write_bytes_per_launch'] = 1024.0 * sum(w) / len(w)
    if 'read_bytes_per_launch' in res and 'write_bytes_per_launch' in res:
        res['hbm_bytes_per_launch'] = res['read_bytes_per_launch'] + res['write_bytes_per_launch']
    # every propagate-path kernel: total HBM bytes over the pass, by role
    res['by_kernel'] = {}
    for name in sorted(set(fetch) | set(write)):
        if 'propagate' not in name and 'trace' not in name and 'scan' not in name and 'bin_' not in name:
            continue
        res['by_kernel'][name] = {'launches': len(fetch.get(name, [])),
                                  'read_bytes_total': 2.0 * 1024.0 * sum(fetch.get(name, [])),
                                  'write_bytes_total': 1024.0 * sum(write.get(name, []))}
    # L2 hit rate per kernel (TCC_HIT_sum / (HIT + MISS)) over the launches that
    # did work (>= 1e5 L2 requests: the slots that exited at once are excluded)
    hit = per_kernel(os.path.join(d, 'l2'), 'TCC_HIT_sum')
    miss = per_kernel(os.path.join(d, 'l2'), 'TCC_MISS_sum')
    if hit:
        res['l2_hit_rate'] = {}
        res['l2_requests'] = {}
        for name in sorted(set(hit) & set(miss)):
            pairs = [(h, m) for h, m in zip(hit[name], miss[name]) if h + m >= 1e5]
            if not pairs:
                continue
            h, m = sum(p[0] for p in pairs), sum(p[1] for p in pairs)
            res['l2_hit_rate'][name] = h / (h + m)
            res['l2_requests'][name] = {'launches': len(pairs), 'hit': h, 'miss': m}
    # the stamp: kernel sources of this tree (bench.py kernel_source_sha) and the commit
    spec = importlib.util.spec_from_file_location('bench_stamp', os.path.join(ROOT, 'bench.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    res['kernel_source_sha'] = mod.kernel_source_sha()
    res['commit'] = os.environ.get('GIT_HEAD', 'unknown')
    # the workload the passes ran (bench.py only uses a summary of its own workload)
    try:
        with open(os.path.join(d, 'bench_fetch.json')) as f:
            cfg = json.loads(f.read().strip().splitlines()[-1])['config']
        res['workload'] = {'detector': cfg['detector'], 'photons': cfg['photons_per_gpu'],
                           'max_steps': cfg.get('max_steps')}
    except (OSError, ValueError, KeyError, IndexError):
        pass
    res['source'] = 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of bench.py (tools/rocprof_bench.sh), ' + \
        os.path.basename(os.path.normpath(d))
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
