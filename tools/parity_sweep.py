#!/usr/bin/env python3
"""Dev tool (GPU box): photon-by-photon parity of the bench workload against the
oracle on several photon seeds -- the bench's own parity check (bench.py
gpu_sample / _oracle_batches / compare: two pipelined batches, the bench's RNG
slots and launch shape) repeated on fresh isotropic samples, to look for rare
walk decisions (float false positives) beyond the bench's one seed.

usage: tools/parity_sweep.py SEED[,SEED...] [bench.py args, e.g. --photons 10000000]
Prints one JSON line per seed and a summary line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from chroma.photon_source import isotropic
    seeds = [int(s) for s in sys.argv[1].split(',')]
    args = bench.parse_args(sys.argv[2:])
    torch.cuda.set_device(0)
    wl = bench.PropagateWorkload(args, 0, 1, 0, None, args.photons)
    threads = bench.usable_cpus()
    total = bad = 0
    for seed in seeds:
        t0 = time.time()
        wl.photons = isotropic(args.photons, seed=seed)
        n = args.photons
        hosts, _, dt = wl._oracle_batches(n, threads)
        par = wl.compare(wl.gpu_sample(n, args.pipeline), hosts)
        total += n
        bad += 0 if par['ok'] else 1
        keep = ('n', 'ok', 'bit_identical', 'flags_mismatches', 'last_hit_mismatches', 'max_rel', 'stack_overflows')
        out = {k: par[k] for k in keep}
        out.update(seed=seed, oracle_s=round(dt, 1), s=round(time.time() - t0, 1))
        if not par['bit_identical']:
            out['floats'] = {f: v for f, v in par['floats'].items() if v.get('differing')}
            out['first_discrete_mismatches'] = par.get('first_discrete_mismatches')
        print(json.dumps(out), flush=True)
    print(json.dumps({'seeds': seeds, 'photons': total, 'seeds_failed': bad}))


if __name__ == '__main__':
    main()
