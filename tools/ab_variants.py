#!/usr/bin/env python
"""A/B the propagate-kernel variants (CHR_PROPAGATE_VARIANT) in ONE process,
interleaved rounds (cdna_hip_programming.md 5.4 rule 24).  Checks that every
variant gives identical photon histories, last-hit triangles and positions.  Dev tool, not part of the product."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--detector', default='demo')
    ap.add_argument('--photons', type=int, default=4_000_000)
    ap.add_argument('--variants', default='0,1,2,3,4,5,6')
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--max-steps', type=int, default=1000)
    args = ap.parse_args()
    import torch
    import bench
    from chroma import gpu
    from chroma.gpu import gpuarray as ga
    from chroma.photon_source import isotropic
    from types import SimpleNamespace
    torch.cuda.set_device(0)
    det = bench.build_geometry(args.detector, '/tmp/chroma_bench_cache')
    t0 = time.time()
    gdet = gpu.GPUDetector(det)
    print('geometry on device in %.1fs' % (time.time() - t0), flush=True)
    photons = isotropic(args.photons, seed=20260102)
    pristine = SimpleNamespace(pos=ga.to_gpu(gpu.to_float3(photons.pos)), dir=ga.to_gpu(gpu.to_float3(photons.dir)),
                               pol=ga.to_gpu(gpu.to_float3(photons.pol)), wavelengths=ga.to_gpu(photons.wavelengths),
                               t=ga.to_gpu(photons.t), flags=ga.to_gpu(photons.flags), evidx=ga.to_gpu(photons.evidx),
                               true_nphotons=args.photons)
    variants = args.variants.split(',')   # "<n>[:chunked]"
    times = {v: [] for v in variants}
    kms = {v: [] for v in variants}
    ref_flags = None
    for r in range(args.rounds + 1):
        for v in variants:
            opts = v.split(':')
            os.environ['CHR_PROPAGATE_VARIANT'] = opts[0]
            os.environ['CHR_STEP_LAUNCH'] = '0' if 'chunked' in opts[1:] else '1'
            rng = gpu.get_rng_states(512 * 1024, seed=1)
            gp = gpu.GPUPhotons(pristine, copy_flags=True, copy_triangles=False, copy_weights=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gp.propagate(gdet, rng, nthreads_per_block=512, max_blocks=1024, max_steps=args.max_steps)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print('  round %d variant %s: %.1f ms' % (r, v, 1e3 * dt), flush=True)
            fl = (gp.flags.get(), gp.last_hit_triangles.get(), gp.pos.get().view(np.uint32).reshape(len(fl0 := gp.flags.get()), -1))
            if ref_flags is None:
                ref_flags = fl
            else:
                bad = (fl[0] != ref_flags[0]) | (fl[1] != ref_flags[1]) | (fl[2] != ref_flags[2]).any(axis=1)
                if bad.any():
                    print('VARIANT %s DIFFERS from variant %s on %d photons (first %s)' % (
                        v, variants[0], int(bad.sum()), np.flatnonzero(bad)[:8]), flush=True)
            st = gp.last_stats
            if r == 0 and st.nodes_visited:
                n = float(args.photons)
                print('variant %s counters: nodes/photon %.2f tris/photon %.2f walks/photon %.3f  SIMD efficiency '
                      'nodes %.3f tris %.3f  (wave node steps %d, wave tri steps %d)' % (
                          v, st.nodes_visited / n, st.triangles_tested / n, st.traversals / n,
                          st.nodes_visited / (64.0 * max(1, st.wave_node_steps)),
                          st.triangles_tested / (64.0 * max(1, st.wave_triangle_steps)),
                          st.wave_node_steps, st.wave_triangle_steps), flush=True)
                print('variant %s time split: fill_state (traversal) %.1f%% of photon-loop wave cycles' % (
                    v, 100.0 * st.wave_fill_cycles / max(1, st.wave_step_cycles)), flush=True)
            if r > 0:
                times[v].append(dt)
                kms[v].append(gp.last_stats.kernel_ms)
    for v in variants:
        if not times[v]:
            continue
        print('variant %s: wall %.1f ms (min %.1f)  kernel %.1f ms  -> %.1f Mphotons/s' % (
            v, 1e3 * np.median(times[v]), 1e3 * min(times[v]), np.median(kms[v]),
            args.photons / np.median(times[v]) / 1e6), flush=True)


if __name__ == '__main__':
    main()
