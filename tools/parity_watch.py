#!/usr/bin/env python3
"""Dev tool (GPU box, CHROMA_DEVICE_PROFILE=1): follow one photon of the bench's
parity sample step by step on both sides.  The bench's two-batch sample
(bench.py gpu_sample / _oracle_batches: same photons, RNG slots and launch
shape) is propagated on the GPU with the photon watch on (chr_watch_set) and by
the oracle with its watch on (oracle.Watch); every step's ray is then walked
again by the oracle's reference DFS (oracle.intersect_rays) and by the GPU's
lone and pair walkers (chr_walk_lone_timing), so a step whose walk differs is
named with the walker that disagrees.

usage: tools/parity_watch.py SAMPLE_INDEX [bench.py args, e.g. --parity-photons 9897030]
Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

FIELDS = ('kind', 'q_or_step', 'tri', 'dist', 'pos_in', 'dir_in', 'last_in', 'material1', 'abs_len', 'scat_len',
          'pos_out', 'history', 'time_out', 'slot')


def decode(rec):
    r = np.asarray(rec, np.uint32)
    f = r.view(np.float32)
    i = r.view(np.int32)
    return {'kind': int(r[0]), 'q_or_step': int(r[1]), 'tri': int(i[2]), 'dist': float(f[3]),
            'pos_in': f[4:7].tolist(), 'dir_in': f[7:10].tolist(), 'last_in': int(i[10]), 'material1': int(i[11]),
            'abs_len': float(f[12]), 'scat_len': float(f[13]), 'pos_out': f[14:17].tolist(),
            'history': int(r[17]), 'time_out': float(f[18]), 'slot': int(r[19])}


EVENT_KINDS = {1: 'start', 2: 'pop', 3: 'node', 4: 'tri_fetch', 5: 'tri_hit', 6: 'leaf_box', 7: 'drain',
               8: 'drain_publish', 9: 'publish'}
# which words of each event kind are floats
EVENT_FLOATS = {1: (5, 6, 7), 2: (2, 3), 3: (3, 6), 4: (3,), 5: (3, 5), 6: (4, 5), 7: (3,), 8: (3,), 9: (3,)}


def decode_event(e):
    e = np.asarray(e, np.uint32)
    k = int(e[0])
    f = e.view(np.float32)
    return [EVENT_KINDS.get(k, k)] + [float(f[i]) if i in EVENT_FLOATS.get(k, ()) else int(e[i]) for i in range(1, 8)]


def main():
    import ctypes
    import torch
    import bench
    import oracle
    from chroma import gpu
    from chroma.event import Photons
    from chroma.gpu import _native, gpuarray as ga, wide_bvh
    from chroma.gpu.tools import current_stream
    if not _native.lib().chr_device_profile_enabled():
        raise SystemExit('run with CHROMA_DEVICE_PROFILE=1 (the photon watch is in the profile build)')
    index = int(sys.argv[1])
    args = bench.parse_args(sys.argv[2:])
    torch.cuda.set_device(0)
    wl = bench.PropagateWorkload(args, 0, 1, 0, None, args.photons)
    n = min(wl.nphotons, args.parity_photons or wl.nphotons)
    cuts = [0, n // 2, n]
    b = int(np.searchsorted(cuts, index, side='right')) - 1
    local = index - cuts[b]
    out = {'index': index, 'n': n, 'batch': b, 'index_in_batch': local}

    # GPU: gpu_sample's two batches, the watch on batch b's photon
    ph = wl.photons
    gps = [gpu.GPUPhotons(Photons(ph.pos[lo:hi], ph.dir[lo:hi], ph.pol[lo:hi], ph.wavelengths[lo:hi]),
                          copy_flags=True, copy_triangles=False, copy_weights=False)
           for lo, hi in zip(cuts[:-1], cuts[1:])]
    rng = gpu.get_rng_states(wl.nslots, seed=args.seed, first_subsequence=bench.rng_first_subsequence(0, wl.nslots))
    kw = dict(nthreads_per_block=args.nthreads_per_block, max_blocks=args.max_blocks, max_steps=args.max_steps)
    _native.call('chr_watch_set', local, gps[b].pos.gpudata)
    wray = os.environ.get('WATCH_RAY')   # "x,y,z": log trace_kernel's walk of the ray with this origin
    if wray:
        org = np.array([float(v) for v in wray.split(',')], np.float32)
        _native.call('chr_watch_ray', org.ctypes.data, None, 0, None)
    t0 = time.time()
    if args.pipeline:
        gpu.propagate_batches(gps, wl.gdet, rng, **kw)
    else:
        for gp in gps:
            gp.propagate(wl.gdet, rng, **kw)
    torch.cuda.synchronize()
    buf = np.zeros((4096, 20), np.uint32)
    cnt = ctypes.c_uint32(0)
    _native.call('chr_watch_fetch', buf.ctypes.data, 4096, ctypes.byref(cnt))
    gsteps = [decode(r) for r in buf[:min(cnt.value, 4096)]]
    if wray:
        ev = np.zeros((8192, 8), np.uint32)
        ne = ctypes.c_uint32(0)
        _native.call('chr_watch_ray', None, ev.ctypes.data, 8192, ctypes.byref(ne))
        out['walk_events_count'] = ne.value
        out['walk_events'] = [decode_event(e) for e in ev[:min(ne.value, 8192)]]
    got = gps[b].get()
    out['gpu'] = {'seconds': round(time.time() - t0, 1), 'steps': len(gsteps),
                  'final': {'pos': got.pos[local].tolist(), 't': float(got.t[local]),
                            'flags': int(got.flags[local]), 'last_hit': int(got.last_hit_triangles[local])}}

    # oracle: _oracle_batches' two batches, the watch on batch b
    from chroma.gpu.packing import PackedGeometry
    packed = PackedGeometry(wl.det)
    hosts = [oracle.HostPhotons(Photons(ph.pos[lo:hi], ph.dir[lo:hi], ph.pol[lo:hi], ph.wavelengths[lo:hi]))
             for lo, hi in zip(cuts[:-1], cuts[1:])]
    st = oracle.rng_init(wl.nslots, seed=args.seed, first_subsequence=bench.rng_first_subsequence(0, wl.nslots))
    t0 = time.time()
    w = None
    for i, h in enumerate(hosts):
        if i == b:
            w = oracle.Watch(local)
        oracle.propagate(packed, h, st, wl.nslots, args.nthreads_per_block, args.max_blocks, args.max_steps,
                         threads=bench.usable_cpus())
        if i == b:
            osteps = [decode(r) for r in w.records()]
            oracle.Watch.off()
    h = hosts[b]
    out['oracle'] = {'seconds': round(time.time() - t0, 1), 'steps': len(osteps),
                     'final': {'pos': h.pos[local].tolist(), 't': float(h.t[local]), 'flags': int(h.flags[local]),
                               'last_hit': int(h.last_hit_triangles[local])}}
    # whole-sample comparison (is the mismatch reproduced by this build?)
    gall = [gp.get() for gp in gps]
    diff = np.zeros(n, bool)
    for f in ('pos', 'dir', 'pol', 't', 'wavelengths', 'flags', 'last_hit_triangles'):
        ga_ = np.concatenate([getattr(o, f) for o in gall])
        ho_ = np.concatenate([getattr(o, f) for o in hosts])
        d = ga_ != ho_
        diff |= d.any(axis=1) if d.ndim > 1 else d
    out['differing_photons'] = [int(i) for i in np.flatnonzero(diff)[:32]]

    # every step's ray walked again: oracle DFS on the GPU's rays and on its own,
    # the GPU's lone / pair walkers on both
    rays = []
    for side, steps in (('gpu', gsteps), ('oracle', osteps)):
        for k, s in enumerate(steps):
            rays.append((side, k, s['pos_in'], s['dir_in'], s['last_in']))
    if rays:
        o = np.array([r[2] for r in rays], np.float32)
        d = np.array([r[3] for r in rays], np.float32)
        last = np.array([r[4] for r in rays], np.int32)
        odist, otri = oracle.intersect_rays(packed, o, d, last)
        wide, _ = wide_bvh.obtain(wl.det.bvh, wl.gdet.packed)
        rec_id = np.asarray(wide.rec_id)
        rr = np.zeros((len(rays), 7), np.float32)
        rr[:, 0:3] = o
        rr[:, 3:6] = d
        rr[:, 6] = last.view(np.float32)
        dr = ga.to_gpu(rr.reshape(-1))
        walkers = {}
        for walker, name in ((0, 'lone'), (1, 'pair')):
            res = ga.zeros(len(rays) * 4 + 1, np.uint32)
            _native.call('chr_walk_lone_timing', wl.gdet._handle, dr.gpudata, len(rays), 1, 64, walker, res.gpudata,
                         current_stream())
            torch.cuda.synchronize()
            raw = res.get()
            recs = raw[:-1].reshape(len(rays), 4)[:, 0].view(np.int32)
            walkers[name] = [int(rec_id[r]) if r >= 0 else -1 for r in recs]
            walkers[name + '_overflow_word'] = int(raw[-1])
        out['rewalk'] = []
        for j, (side, k, _, _, _) in enumerate(rays):
            steps = gsteps if side == 'gpu' else osteps
            out['rewalk'].append({'side': side, 'step': k, 'recorded_tri': steps[k]['tri'],
                                  'recorded_dist': steps[k]['dist'], 'oracle_tri': int(otri[j]),
                                  'oracle_dist': float(odist[j]), 'lone_tri': walkers['lone'][j],
                                  'pair_tri': walkers['pair'][j]})
        out['walker_overflow_words'] = {k: v for k, v in walkers.items() if k.endswith('_word')}
    out['gpu_steps'] = gsteps
    out['oracle_steps'] = osteps
    print(json.dumps(out))


if __name__ == '__main__':
    main()
