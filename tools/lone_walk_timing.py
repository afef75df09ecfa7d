#!/usr/bin/env python3
"""Dev tool (GPU box): the lone-photon walk (walk_lone) timed in isolation,
chr_walk_lone_timing.  Rays: the photons still alive after 3 steps of a 1 M
isotropic batch on the bench detector (later-step rays, as in the tail).  Each
ray walked `reps` times in a row (the first walk cold, the others with the
path's nodes warm in L2) by 1, 256 and 2048 concurrent waves.  Prints the
median ns / cycles per iteration and per walk."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import torch
    from chroma import gpu
    from chroma.gpu import _native, gpuarray as ga
    from chroma.gpu.tools import current_stream
    from chroma.photon_source import isotropic
    det_name = sys.argv[1] if len(sys.argv) > 1 else '29k'
    torch.cuda.set_device(0)
    det, _ = bench.shared_geometry(det_name, os.environ.get('CHROMA_BENCH_CACHE', '/tmp/chroma_bench_cache'), 0, None)
    gdet = gpu.GPUDetector(det)
    ph = isotropic(1_000_000, seed=11)
    gp = gpu.GPUPhotons(ph, copy_flags=True, copy_triangles=False, copy_weights=False)
    rng = gpu.get_rng_states(512 * 1024, seed=1)
    gp.propagate(gdet, rng, nthreads_per_block=512, max_blocks=1024, max_steps=3)
    got = gp.get()
    alive = np.flatnonzero((got.flags & 0x800F) == 0)[:4096]   # not dead (NO_HIT, ABSORB, DETECT, NAN)
    rays = np.zeros((len(alive), 7), np.float32)
    rays[:, 0:3] = got.pos[alive]
    d = got.dir[alive].astype(np.float64)
    rays[:, 3:6] = (d / np.linalg.norm(d, axis=1)[:, None]).astype(np.float32)
    rays[:, 6] = got.last_hit_triangles[alive].astype(np.int32).view(np.float32)
    dr = ga.to_gpu(rays.reshape(-1))
    reps = 8
    out = {'detector': det_name, 'rays': int(len(alive))}
    base = None
    for walker, wname in ((0, 'lone'), (1, 'pair')):
        for nw in (1, 256, 2048):
            n = len(alive) if nw > 1 else 256
            res = ga.zeros(n * reps * 4 + 1, np.uint32)
            _native.call('chr_walk_lone_timing', gdet._handle, dr.gpudata, n, reps, nw, walker, res.gpudata,
                         current_stream())
            torch.cuda.synchronize()
            raw = res.get()
            r = raw[:-1].reshape(n, reps, 4).astype(np.float64)
            it = np.maximum(r[:, :, 1], 1)
            row = {}
            for name, sl in (('first', slice(0, 1)), ('warm', slice(1, reps))):
                row[name] = {'iterations': float(np.median(r[:, sl, 1])),
                             'ns_per_walk': float(np.median(r[:, sl, 2] * 10)),
                             'ns_per_iteration': float(np.median(r[:, sl, 2] * 10 / it[:, sl])),
                             'cycles_per_iteration': float(np.median(r[:, sl, 3] / it[:, sl]))}
            same = bool(np.all(r[:, :, 0] == r[:, :1, 0]))
            tris = raw[:-1].reshape(n, reps, 4)[:, 0, 0]
            if nw == 2048:
                if walker == 0:
                    base = tris.copy()
                else:
                    row['same_as_lone'] = bool(np.array_equal(tris, base[:len(tris)]))
            row['overflow'] = int(raw[-1])
            out['%s_waves_%d' % (wname, nw)] = dict(row, results_repeat=same, rays=n)
            print(json.dumps({'walker': wname, 'waves': nw, **row}), flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
