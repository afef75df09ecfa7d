#!/usr/bin/env python
"""SURVEY §8(d) algorithmic bytes per photon, per benchmark configuration:
the CPU oracle walks the REFERENCE BVH (recursive grid, degree 3) in the
reference traversal order (mesh.h:75-117) on a 10^5-photon subsample of each
config's input (the first photons of bench.py's isotropic source, bench.py's
launch shape), counting nodes box-tested, triangles tested and walks:

    B_alg = 120 + (16 N_node + 48 N_tri + 4 N_walk) / photons   [bytes/photon]

usage: python tools/bytes_per_photon.py [--configs tiny,demo,scint,29k] > profiles/bytes_per_photon.json
(geometry cached under --cache-dir like bench.py)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

import bench  # noqa: E402  (detector table, geometry cache, photon seed, launch shape)

# BASELINE.json configs: photons of each benchmark input
CONFIG_PHOTONS = {'tiny': 1_000_000, 'demo': 10_000_000, 'scint': 10_000_000, '29k': 10_000_000}
CONFIG_NAME = {'tiny': 'C2 demo.tiny()', 'demo': 'C3 demo.detector()', 'scint': 'C5 demo.scint.detector()',
               '29k': 'bench / north star: 29k-PMT detector'}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='tiny,demo,scint,29k')
    ap.add_argument('--photons', type=int, default=100_000)
    ap.add_argument('--max-steps', type=int, default=1000)
    ap.add_argument('--nthreads-per-block', type=int, default=512)
    ap.add_argument('--max-blocks', type=int, default=1024)
    ap.add_argument('--threads', type=int, default=os.cpu_count() or 1)
    ap.add_argument('--cache-dir', default=os.environ.get('CHROMA_BENCH_CACHE', '/tmp/chroma_bench_cache'))
    args = ap.parse_args()
    import oracle
    from chroma.event import Photons
    from chroma.gpu.packing import PackedGeometry
    from chroma.photon_source import isotropic
    out = {'definition': 'B_alg = 120 + (16*N_node + 48*N_tri + 4*N_walk)/photons; N counted by the CPU oracle on '
                         'the reference BVH (recursive grid, degree 3) in reference order (SURVEY 8(d))',
           'launch_shape': [args.nthreads_per_block, args.max_blocks], 'max_steps': args.max_steps,
           'photon_seed': bench.PHOTON_SEED, 'configs': {}}
    for name in args.configs.split(','):
        t0 = time.time()
        det = bench.build_geometry(name, args.cache_dir)
        packed = PackedGeometry(det)
        src = isotropic(CONFIG_PHOTONS[name], seed=bench.PHOTON_SEED)
        n = min(args.photons, CONFIG_PHOTONS[name])
        sample = Photons(src.pos[:n], src.dir[:n], src.pol[:n], src.wavelengths[:n])
        host = oracle.HostPhotons(sample)
        nslots = args.nthreads_per_block * args.max_blocks
        st = oracle.rng_init(nslots, seed=1)
        t1 = time.time()
        s = oracle.propagate(packed, host, st, nslots, args.nthreads_per_block, args.max_blocks, args.max_steps,
                             threads=args.threads)
        dt = time.time() - t1
        walks = s['traversals']
        b = 120.0 + (16.0 * s['nodes_visited'] + 48.0 * s['tris_tested'] + 4.0 * walks) / n
        out['configs'][name] = {
            'config': CONFIG_NAME[name], 'geometry': bench.DETECTORS[name][0],
            'triangles': int(len(det.mesh.triangles)), 'reference_bvh_nodes': int(len(det.bvh.nodes)),
            'input_photons': CONFIG_PHOTONS[name], 'sample_photons': n,
            'nodes_visited': s['nodes_visited'], 'triangles_tested': s['tris_tested'], 'walks': walks,
            'walks_per_photon': walks / n, 'nodes_per_walk': s['nodes_visited'] / max(1, walks),
            'triangles_per_walk': s['tris_tested'] / max(1, walks),
            'bytes_per_walk': (16.0 * s['nodes_visited'] + 48.0 * s['tris_tested'] + 4.0 * walks) / max(1, walks),
            'bytes_per_photon': b, 'max_stack_depth': s['max_depth'], 'stack_overflows': s['overflows'],
            'oracle_seconds': round(dt, 2), 'oracle_threads': args.threads}
        print('%s: %.0f B/photon, %.2f walks/photon, %.1f nodes + %.1f triangles per walk (%.1fs, build %.1fs)' % (
            name, b, walks / n, s['nodes_visited'] / max(1, walks), s['tris_tested'] / max(1, walks), dt,
            t1 - t0), file=sys.stderr, flush=True)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main()
