#!/usr/bin/env python
"""Per-photon step profile of a propagate, from the CPU oracle (diagnostics).

Which photons set the length of the multi-step tail launch (photon.py:261-264:
below nthreads_per_block*128 survivors, one launch runs every remaining step)?
Runs oracle.propagate with orc_set_profile on a bench detector and prints the
distribution of steps per photon, the longest-lived photons (steps, reference
BVH nodes per step, final history bits, position), so the tail's serial chain
can be read off without a GPU.

    python tools/tail_profile.py --detector demo --photons 2000000
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
sys.path.insert(0, ROOT)

FLAGS = ['NO_HIT', 'BULK_ABSORB', 'SURFACE_DETECT', 'SURFACE_ABSORB', 'RAYLEIGH_SCATTER', 'REFLECT_DIFFUSE',
         'REFLECT_SPECULAR', 'SURFACE_REEMIT', 'SURFACE_TRANSMIT', 'BULK_REEMIT', 'CHERENKOV', 'SCINTILLATION']


def names(h):
    return '|'.join(n for i, n in enumerate(FLAGS) if h & (1 << i)) + ('|NAN_ABORT' if h & (1 << 15) else '')


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument('--detector', default='demo')
    ap.add_argument('--photons', type=int, default=1_000_000)
    ap.add_argument('--max-steps', type=int, default=1000)
    ap.add_argument('--seed', type=int, default=1)
    ap.add_argument('--top', type=int, default=20)
    ap.add_argument('--repeat', type=int, default=1,
                    help='propagates of the same photons with the RNG states carried on (bench.py steps)')
    ap.add_argument('--cache-dir', default='/tmp/chroma_bench_cache')
    args = ap.parse_args()
    import bench
    import oracle
    from chroma.event import Photons
    from chroma.gpu.packing import PackedGeometry
    from chroma.photon_source import isotropic
    det = bench.build_geometry(args.detector, args.cache_dir)
    packed = PackedGeometry(det)
    src = isotropic(args.photons, seed=bench.PHOTON_SEED)
    nslots = 512 * 1024
    st = oracle.rng_init(nslots, seed=args.seed)
    oracle.lib().orc_set_profile.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for rep in range(args.repeat):
        host = oracle.HostPhotons(Photons(src.pos, src.dir, src.pol, src.wavelengths))
        steps = np.zeros(args.photons, np.uint32)
        nodes = np.zeros(args.photons, np.uint32)
        oracle.lib().orc_set_profile(steps.ctypes.data, nodes.ctypes.data)
        t0 = time.time()
        stats = oracle.propagate(packed, host, st, nslots, 512, 1024, args.max_steps)
        oracle.lib().orc_set_profile(None, None)
        print('propagate %d: %.1fs, host steps %d, stats %s' % (rep, time.time() - t0, stats['host_steps'], stats))
        q = [50, 90, 99, 99.9, 99.99, 100]
        print('steps per photon percentiles', dict(zip(q, np.percentile(steps, q))))
        order = np.argsort(steps)[::-1][:args.top]
        for i in order:
            print('photon %8d steps %4d nodes/step %7.1f flags %-60s pos %s r %.0f' % (
                i, steps[i], nodes[i] / max(1, steps[i]), names(int(host.flags[i])), np.round(host.pos[i], 1),
                np.linalg.norm(host.pos[i])))
        worst = np.argsort(nodes)[::-1][:5]
        print('most nodes:', [(int(i), int(steps[i]), int(nodes[i])) for i in worst])
        sys.stdout.flush()


if __name__ == '__main__':
    main()
