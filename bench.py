#!/usr/bin/env python
"""Benchmark: propagated photons/s of GPUPhotons.propagate (the reference's
hot path, chroma/gpu/photon.py:226-293) on a demo PMT detector.

One "step" = one propagate of a fresh batch of isotropic photons (BASELINE.md
section 3 source: centre point source, seed 20260102+rank) to termination or
max_steps (default 1000, the Simulation.simulate default), launch shape of
Simulation (nthreads_per_block=512, max_blocks=1024 -> 524,288 RNG slots).
Photon inputs are resident in HBM before the timed region; each step restores
them from a device-resident copy (D2D, inside the timed region).

Steps are pipelined (default; --no-pipeline for one synchronous propagate per
step): up to --pipeline-depth steps go to one chroma.gpu.propagate_batches
call, which propagates them in order with the one rng_states exactly as that
many propagate calls would (bit-identical photons and RNG states, tested in
tests/test_gpu_batches.py) while each batch's multi-step tail -- as long as
its longest-lived photon's serial chain -- runs on a second HIP stream under
the next batch's first-step queueing, binning and BVH walk (which draw no
random numbers).  detail.step_ms is then each call's time split over its
steps.  A short sequential run of the same steps follows, untimed for the
headline, and is reported as detail.sequential (the figure a caller making one
propagate call at a time gets).

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) this process
is one rank; with --gpus N > 1 and no WORLD_SIZE, bench.py starts the N rank
processes itself (before touching any GPU) and exits with the first failing
rank's status.  The geometry is replicated, the photons sharded: --photons
per GPU (weak scaling, the default) or --total-photons over all GPUs (strong
scaling; C4 is --gpus 8 --total-photons 100000000).  Each rank draws disjoint
RNG subsequences (rank*nslots + slot).  Each step ends with the hit-channel
reduce: detected photons are histogrammed per PMT channel on the device and
SUM-reduced over the ranks (RCCL, chroma.gpu.shard) -- the only exchange the
path has.  The timed region is bracketed by barriers and the max over ranks
is reported; value = photons of all ranks / that time.

Parity: rank 0 runs the CPU oracle (cpu_baseline leg, the only place bench.py
touches oracle/) on a bounded sample of its photons with the same RNG
initialisation, as two batches in order, then propagates the SAME two batches
on the GPU through the path the headline used (pipelined or sequential) and
compares photon by photon (history flags, last-hit triangles and channels
bit-exact; positions, directions, polarisations, times and wavelengths as a
max relative difference).  Ranks > 0 propagate a smaller sample of their own
shard (their own photon seed and RNG subsequences) on their GPU and send the
photons to rank 0, which runs the oracle for them: parity.per_rank (only rank
0 holds the oracle's host copy of the geometry).  detail.ranks carries each
rank's setup times (geometry build / cache load, upload) and host memory.

Roofline: the dominant kernel is trace_kernel, the
BVH walk of every one-step launch.  It is bound by HBM/L2 latency-bandwidth on
dependent node/triangle gathers.
    achieved = algorithmic bytes per trace launch / average trace launch time
with the average from HIP events around each trace launch on its stream, and
the algorithmic bytes of section 8(d): per walk 16 * reference-BVH nodes +
48 * reference triangles + 4, counted by the CPU oracle walking the REFERENCE
BVH in the reference's DFS order on the cpu_baseline sample of the same
workload, times the rays of the launch.  Every rank reports its own launches
(roofline.per_rank).  traffic = HBM bytes per trace launch from the rocprofv3
FETCH_SIZE/WRITE_SIZE passes of this workload and l2_hit_rate from its
TCC_HIT/TCC_MISS pass; those counters cannot be read from inside this
process, so they are copied from profiles/latest_pmc.json, which is stamped
with the sha of the kernel sources it measured: a stamp that differs from
this tree's sources is reported as stale.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))

import numpy as np  # noqa: E402

METRIC = 'propagated photons/sec, 29k-PMT detector, 10M isotropic photons, 1/2/4/8 GPUs'
HBM_PEAK_GBS = 8000.0
PHOTON_SEED = 20260102
PUBLISHED_29K = 2.5e6      # reference README, 29k PMTs, photons/s


def _demo_detector(**kw):
    from chroma import demo
    return demo.detector(**kw)


def _scint_detector(**kw):
    from chroma.demo import scint
    return scint.detector(**kw)


DETECTORS = {
    # name: (description, kwargs, builder)
    '29k': ('demo.detector(pmt_radius=23780, sphere_radius=24280): 29,007 PMTs, ~170M triangles',
            dict(pmt_radius=23780.0, sphere_radius=24280.0), _demo_detector),
    'demo': ('demo.detector(): 10,055 PMTs, 58.96M triangles', dict(), _demo_detector),
    'tiny': ('demo.tiny(): 53 PMTs, 389,568 triangles', dict(pmt_radius=2000.0, sphere_radius=2500.0,
                                                             spiral_step=700.0), _demo_detector),
    'small': ('demo.detector(600, 900, 1500): 2 PMTs, 90,912 triangles',
              dict(pmt_radius=600.0, sphere_radius=900.0, spiral_step=1500.0), _demo_detector),
    # BASELINE config 5: scintillator + WLS + dichroic surfaces (chroma.demo.scint)
    'scint': ('demo.scint.detector(): 10,055 PMTs in liquid scintillator (2-component bulk re-emission), '
              'light cones cycling shiny / dichroic / WLS, 58.96M triangles', dict(), _scint_detector),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def usable_cpus():
    """Host cores this job may use: the affinity mask, capped by a cgroup CPU
    quota (a GPU box shares its host: nproc shows every core of the machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            quota, period = f.read().split()[:2]
        if quota != 'max':
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def host_memory():
    """This process's host memory: resident now and its peak (GB), from
    /proc/self/status (a replicated 29k geometry is ~15 GB of host memory per rank)."""
    out = {}
    try:
        with open('/proc/self/status') as f:
            for line in f:
                k, _, v = line.partition(':')
                if k in ('VmRSS', 'VmHWM'):
                    out['host_rss_gb' if k == 'VmRSS' else 'host_peak_rss_gb'] = round(int(v.split()[0]) / 1e6, 3)
    except (OSError, ValueError):
        pass
    return out


def kernel_source_sha():
    """sha256 (16 hex) of the sources libchroma_amd.so is built from
    (tools/source_sha.py): the stamp that ties a committed PMC record to the
    kernels it measured."""
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    from source_sha import kernel_source_sha as sha
    return sha(ROOT)


def so_source_sha():
    """The sha compiled into the loaded libchroma_amd.so (chr_source_sha): the
    library travels prebuilt with the tree, so the line says whether it was
    built from these sources."""
    from chroma.gpu import _native
    try:
        return _native.lib().chr_source_sha().decode()
    except (AttributeError, OSError, _native.NativeError) as e:   # an older library
        return 'unavailable: %s' % e


def build_geometry(name, cache_dir):
    """Flattened demo detector + BVH, cached on local disk (same box reuse)."""
    from chroma.bvh import make_recursive_grid_bvh
    from chroma.cache import Cache
    t0 = time.time()
    cache = None
    if cache_dir:
        try:
            os.makedirs(cache_dir, exist_ok=True)
            cache = Cache(cache_dir)
        except OSError as e:
            log('geometry cache unavailable: %s' % e)
    key = 'bench_%s' % name
    if cache is not None and key in cache.list_geometry():
        det = cache.load_geometry(key)
        det.bvh = cache.load_bvh(cache.get_geometry_hash(key))
        log('geometry %s loaded from cache in %.1fs' % (name, time.time() - t0))
        return det
    det = DETECTORS[name][2](**DETECTORS[name][1])
    det.flatten()
    t1 = time.time()
    det.bvh = make_recursive_grid_bvh(det.mesh, target_degree=3)
    log('geometry %s: %d triangles, flatten %.1fs, BVH %.1fs (%d nodes)' % (
        name, len(det.mesh.triangles), t1 - t0, time.time() - t1, len(det.bvh.nodes)))
    if cache is not None:
        try:
            cache.save_bvh(det.bvh, det.mesh.md5())
            cache.save_geometry(key, det)
        except OSError as e:
            log('geometry cache not written: %s' % e)
    return det


def shared_geometry(name, cache_dir, rank, dist):
    """Rank 0 builds (flatten + BVH: minutes for the 29k detector) and fills
    the node-local cache -- the reference BVH and the traversal BVH derived from
    it (chroma.gpu.wide_bvh, 33-36 s of host build on the 29k detector) -- while
    the other ranks wait at a barrier, then load both from the cache.  Returns
    (geometry, setup phases: geometry_s, and on rank 0 of a multi-rank job
    wide_bvh_prepare_s / wide_bvh_prepare_source)."""
    t0 = time.time()
    if dist is None or not cache_dir:
        return build_geometry(name, cache_dir), {'geometry_s': round(time.time() - t0, 2)}
    setup = {}
    if rank == 0:
        det = build_geometry(name, cache_dir)
        setup['geometry_s'] = round(time.time() - t0, 2)
        from chroma.gpu import wide_bvh
        t1 = time.time()
        setup['wide_bvh_prepare_source'] = wide_bvh.prepare(det)
        setup['wide_bvh_prepare_s'] = round(time.time() - t1, 2)
    dist.barrier()
    if rank != 0:
        t1 = time.time()
        det = build_geometry(name, cache_dir)
        setup['geometry_s'] = round(time.time() - t1, 2)
        setup['barrier_wait_s'] = round(t1 - t0, 2)
    return det, setup


def _native_host_threads():
    from chroma.gpu import _native
    return _native.host_threads()


# Host memory one rank holds (GB), measured on MI355X boxes (profiles/r05: 29k rank 0
# peaks at 63.6 GB with a cold geometry build plus the oracle's parity sample, a rank
# loading geometry and traversal BVH from the node-local cache holds 24.6-25.1 GB):
# (rank 0: build + oracle checks, any other rank: cache load + device upload)
HOST_GB_PER_RANK = {'29k': (64.0, 26.0), 'demo': (28.0, 11.0), 'scint': (28.0, 11.0), 'tiny': (3.0, 2.0),
                    'small': (2.0, 1.0)}


def host_memory_available():
    """Bytes of host memory this job can still take: MemAvailable, capped by the
    cgroup limit (memory.max - memory.current) when one is set.
    CHROMA_BENCH_MEMAVAILABLE_GB overrides (tests)."""
    o = os.environ.get('CHROMA_BENCH_MEMAVAILABLE_GB')
    if o:
        return float(o) * 1e9
    avail = None
    try:
        with open('/proc/meminfo') as f:
            for line in f:
                if line.startswith('MemAvailable:'):
                    avail = int(line.split()[1]) * 1024.0
    except (OSError, ValueError):
        pass
    try:
        with open('/sys/fs/cgroup/memory.max') as f:
            lim = f.read().strip()
        if lim != 'max':
            with open('/sys/fs/cgroup/memory.current') as f:
                room = float(int(lim) - int(f.read().strip()))
            avail = room if avail is None else min(avail, room)
    except (OSError, ValueError):
        pass
    return avail


def preflight_host_memory(detector, local_world, avail=None):
    """Does this node's host memory hold every local rank of the job?  Rank 0
    builds (or loads) the geometry and runs the oracle checks, every other rank
    loads the geometry from the node-local cache and keeps its host copy.
    Returns the record the line carries (detail.preflight); 'fits' False means
    the run is refused before any rank allocates (an out-of-memory kill of 8
    ranks mid-setup would say nothing)."""
    first, other = HOST_GB_PER_RANK.get(detector, (0.0, 0.0))
    need = (first + other * max(0, local_world - 1)) * 1e9
    avail = host_memory_available() if avail is None else avail
    return {'local_ranks': local_world, 'need_gb': round(need / 1e9, 1),
            'per_rank_gb': {'rank0': first, 'other': other},
            'available_gb': None if avail is None else round(avail / 1e9, 1),
            'fits': avail is None or need <= avail}


def rng_first_subsequence(rank, nslots):
    """Rank r's RNG slots are curand subsequences [r*nslots, (r+1)*nslots):
    disjoint streams, and rank 0 draws what a single-GPU run draws."""
    return rank * nslots


def photons_for_rank(args, rank, world):
    """Photons this rank propagates per step: --photons (weak scaling) or its
    contiguous share of --total-photons (strong scaling, chroma.gpu.shard)."""
    if args.total_photons:
        lo, hi = args.total_photons * rank // world, args.total_photons * (rank + 1) // world
        return hi - lo
    return args.photons


def timed_loop(run, steps, warmup, dist, sync, group=1, prepare=None):
    """W untimed steps, then K timed steps bracketed by barrier + sync on both
    sides; run(m) performs m steps and returns their results (m > 1: one
    pipelined call, see main).  prepare(m), when the K steps are one group: the
    steps' input batches filled before the timer starts (inputs resident in HBM
    at t0), instead of by run(m) inside the timed region.  Returns (elapsed max
    over ranks, this rank's per-step seconds -- a group's time split evenly over
    its steps --, per-step results)."""
    if warmup:
        run(warmup)
    if prepare is not None and group >= steps:
        prepare(steps)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    results, per_step = [], []
    left = steps
    while left > 0:
        m = min(group, left)
        t1 = time.perf_counter()
        results.extend(run(m))
        t2 = time.perf_counter()   # the calls are synchronous: a mark per group
        per_step.extend([(t2 - t1) / m] * m)
        left -= m
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = _allreduce(dist, elapsed, 'max')
    return elapsed, per_step, results


def _allreduce(dist, x, op):
    import torch
    dev = 'cuda' if (torch.cuda.is_available() and dist.get_backend() != 'gloo') else 'cpu'
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == 'max' else dist.ReduceOp.SUM)
    return float(t.item())


FLOAT_RTOL = 1e-5
PARITY_RULE = ('flags, last-hit triangles, channels bit-exact; |gpu - oracle| <= 1e-5 * max(|oracle|, 1) per '
               'component for pos (mm), dir, pol, 1e-5 * |oracle| for t and wavelengths (BASELINE north_star, '
               'tests/test_gpu_configs_full.py)')


def photon_record(i, batches, gf, hf, gl, hl):
    """Where photon i of a parity sample sits (batch, index in it) and its
    discrete outcome on both sides."""
    b = int(np.searchsorted(np.cumsum(batches), i, side='right'))
    return {'index': int(i), 'batch': b, 'index_in_batch': int(i - sum(batches[:b])),
            'flags_gpu': int(gf[i]), 'flags_oracle': int(hf[i]),
            'last_hit_gpu': int(gl[i]), 'last_hit_oracle': int(hl[i])}


def float_contract(a, b, field, batches, gf, hf, gl, hl):
    """The float parity rule for one photon field (PARITY_RULE): violation count,
    largest absolute difference, and the worst photon (largest |a-b| / tolerance)
    with its values, flags and last hit."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    floor = 1.0 if field in ('pos', 'dir', 'pol') else 0.0
    tol = FLOAT_RTOL * np.maximum(np.abs(b), floor)
    diff = np.abs(a - b)
    with np.errstate(divide='ignore', invalid='ignore'):
        ratio = np.where(diff == 0, 0.0, np.where(tol > 0, diff / np.where(tol > 0, tol, 1.0), np.inf))
    ratio = np.where(np.isnan(a) & np.isnan(b), 0.0, np.where(np.isnan(ratio), np.inf, ratio))
    if ratio.ndim > 1:
        per_photon = ratio.max(axis=1)
        dmax = diff.max(axis=1)
    else:
        per_photon, dmax = ratio, diff
    out = {'violations': int(np.count_nonzero(per_photon > 1.0)), 'differing': int(np.count_nonzero(dmax > 0)),
           'max_abs': float(np.nanmax(dmax)) if dmax.size else 0.0}
    if dmax.size and out['differing']:
        i = int(np.argmax(per_photon))
        rec = photon_record(i, batches, gf, hf, gl, hl)
        rec.update({'gpu': np.atleast_1d(a[i]).tolist(), 'oracle': np.atleast_1d(b[i]).tolist(),
                    'abs_diff': np.atleast_1d(diff[i]).tolist(), 'over_tolerance': float(per_photon[i])})
        out['worst'] = rec
        out['differing_sample'] = [int(j) for j in np.flatnonzero(dmax > 0)[:16]]
    return out


REFERENCE_GEOMETRY_KEYS = {'29k': 'detector_29k', 'demo': 'demo_detector'}


def geometry_md5_check(name, det, detail):
    """The bench geometry against the reference generator's own build
    (tests/golden/reference_hashes.json, written by make_golden_geometry.py in
    the build container): True / False, or None when no record exists for this
    detector (or the workload has no host geometry).  The hashes go to
    detail.geometry_hashes."""
    key = REFERENCE_GEOMETRY_KEYS.get(name)
    if key is None or det is None or not hasattr(det, 'mesh'):
        return None
    with open(os.path.join(ROOT, 'tests', 'golden', 'reference_hashes.json')) as f:
        want = json.load(f).get(key)
    if want is None:
        return None
    from chroma.demo import geometry_hashes
    t0 = time.time()
    got = geometry_hashes(det)
    fields = sorted(k for k in got if k in want)
    detail['geometry_hashes'] = {'reference_record': 'tests/golden/reference_hashes.json[%s]' % key,
                                 'fields': fields, 'differ': [k for k in fields if got[k] != want[k]],
                                 'seconds': round(time.time() - t0, 1)}
    return not detail['geometry_hashes']['differ']


def result_line(args, world, elapsed, per_step_s, total_photons, detector_info, detail):
    value = total_photons / elapsed
    group = detail.get('pipelined_steps_per_call', 1)
    if args.pipeline and group > 1:
        call = ('chroma.gpu.propagate_batches (the call Simulation.simulate makes) of %d batches per call, '
                'each batch one GPUPhotons.propagate-equivalent of' % group)
    else:
        call = 'one GPUPhotons.propagate call per step of'
    workload = ('%s %s isotropic photons on %s, max_steps=%d, launch shape %dx%d (%d RNG slots)' % (
        call, ('%d in total over %d GPUs' % (args.total_photons, world)) if args.total_photons
        else ('%d per GPU' % args.photons), DETECTORS[args.detector][0], args.max_steps,
        args.nthreads_per_block, args.max_blocks, args.nthreads_per_block * args.max_blocks))
    cfg = {'workload': workload, 'timed_call': 'propagate_batches' if (args.pipeline and group > 1) else 'propagate',
           'batches_per_call': group if args.pipeline else 1,
           'detector': args.detector, 'max_steps': args.max_steps,
           'parallelism': 'photon-sharded x%d, geometry replicated' % world}
    if args.total_photons:
        cfg['total_photons'] = args.total_photons
    else:
        cfg['photons_per_gpu'] = args.photons
    return {
        'metric': METRIC, 'value': value, 'unit': 'photons/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': 1e3 * elapsed / args.steps, 'higher_is_better': True,
        'scaling': 'strong' if args.total_photons else 'weak',
        'vs_baseline': (value / PUBLISHED_29K) if args.detector == '29k' else None,
        'dtype': 'f32', 'data': 'synthetic isotropic point source (BASELINE.md section 3), seed %d+rank' % PHOTON_SEED,
        'config': dict(cfg, **detector_info),
        'value_propagate_per_call': value if not args.pipeline else (detail.get('sequential') or {}).get('photons_per_s'),
        'value_propagate_per_call_note': 'one GPUPhotons.propagate call per step (the reference caller\'s loop, '
                                         'its multi-step tail not overlapped): detail.sequential',
        'detail': dict({'step_ms': [round(1e3 * s, 3) for s in per_step_s]}, **detail),
        'roofline': None, 'cpu_baseline': None, 'parity': None,
    }


def _kernel_info(native):
    try:
        return native.kernel_info()
    except (AttributeError, native.NativeError) as e:     # an older library (A/B runs)
        return 'unavailable: %s' % e


def pmc_record(args):
    """The committed PMC summary of this workload (profiles/latest_pmc.json):
    (record, note) -- note says why it is not used or that it is stale."""
    pmc_path = os.path.join(ROOT, 'profiles', 'latest_pmc.json')
    if not os.path.exists(pmc_path):
        return None, 'no profiles/latest_pmc.json'
    with open(pmc_path) as f:
        pmc = json.load(f)
    w = pmc.get('workload', {})
    if (w.get('detector'), w.get('photons'), w.get('max_steps')) != (args.detector, args.photons, args.max_steps) \
            or pmc.get('kernel') != 'chr::trace_kernel':
        return None, 'profiles/latest_pmc.json measured another workload'
    return pmc, None


def roofline(args, reports, ref):
    """roofline object of the bench line for the dominant kernel (trace_kernel):
    rank 0's launches as the headline, every rank's in per_rank."""
    per_walk = (16.0 * ref['nodes_visited'] + 48.0 * ref['tris_tested']) / ref['traversals'] + 4.0

    def of(rep):
        launches = max(1, rep['trace_launches'])
        rays_per_launch = rep['trace_rays'] / launches
        avg_launch_s = rep['trace_ms'] / launches / 1e3
        alg = rays_per_launch * per_walk
        ach = alg / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
        return alg, rays_per_launch, avg_launch_s, ach

    r0 = reports[0]
    alg, rays_per_launch, avg_launch_s, achieved = of(r0)
    lm = np.asarray(r0['launch_ms'], np.float64)
    rl = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
          'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
          'kernel': 'chr::trace_kernel (BVH walk of the one-step launches)',
          'basis': 'SURVEY 8(d): 16 B x reference-BVH nodes + 48 B x triangles + 4 B per walk '
                   '(oracle, reference DFS order, on the cpu_baseline sample)',
          'alg_bytes_per_launch': alg, 'alg_bytes_per_walk': per_walk,
          'rays_per_launch': rays_per_launch, 'avg_launch_ms': 1e3 * avg_launch_s,
          'launches_timed': r0['trace_launches'],
          'launch_ms_min': float(lm.min()) if lm.size else None,
          'launch_ms_median': float(np.median(lm)) if lm.size else None,
          'launch_ms_max': float(lm.max()) if lm.size else None,
          'reference_bvh_nodes_per_walk': ref['nodes_visited'] / ref['traversals'],
          'reference_bvh_triangles_per_walk': ref['tris_tested'] / ref['traversals'],
          'l2_hit_rate': None}
    if len(reports) > 1:
        rl['per_rank'] = []
        for rep in reports:
            a, rpl, avg, ach = of(rep)
            rl['per_rank'].append({'rank': rep['rank'], 'avg_launch_ms': 1e3 * avg, 'rays_per_launch': rpl,
                                   'launches_timed': rep['trace_launches'], 'achieved': ach,
                                   'frac': ach / HBM_PEAK_GBS})
    pmc, note = pmc_record(args)
    sha = kernel_source_sha()
    rl['kernel_source_sha'] = sha
    rl['so_source_sha'] = so_source_sha()
    rl['so_built_from_these_sources'] = rl['so_source_sha'] == sha
    if pmc is None:
        rl['traffic_source'] = note
        return rl
    stamp = pmc.get('kernel_source_sha')
    stale = stamp != sha
    if 'hbm_bytes_per_launch' in pmc:
        rl['traffic'] = pmc['hbm_bytes_per_launch']
        rl['traffic_unit'] = 'bytes/launch (FETCH_SIZE x2 + WRITE_SIZE)'
    l2 = pmc.get('l2_hit_rate', {}).get('chr::trace_kernel')
    if l2 is not None:
        rl['l2_hit_rate'] = l2
    rl['traffic_source'] = '%s: profiles/latest_pmc.json (%s; commit %s, kernel_source_sha %s%s)' % (
        'STALE (kernel sources changed since the PMC passes)' if stale else 'copied, same kernel sources',
        pmc.get('source'), pmc.get('commit'), stamp,
        '' if not stale else ' != this tree %s' % sha)
    rl['traffic_stale'] = stale
    return rl


class PropagateWorkload(object):
    """One rank's share of the bench: geometry on its GPU, its photon batches
    resident in HBM, and the steps.  bench.py's rank logic (timing, reduces,
    the line) only calls the methods below."""

    def __init__(self, args, rank, world, local, dist, nphotons):
        import torch
        from chroma import gpu
        from chroma.gpu import gpuarray as ga
        from chroma.photon_source import isotropic
        from types import SimpleNamespace
        self.args, self.rank, self.world, self.local, self.nphotons = args, rank, world, local, nphotons
        self.torch = torch
        t_setup = time.time()
        self.det, self.setup = shared_geometry(args.detector, args.cache_dir, rank, dist)
        t0 = time.time()
        self.gdet = gpu.GPUDetector(self.det)
        # GPUDetector's phases: packing, traversal BVH (cache load or host build), H2D
        self.setup['upload_s'] = round(time.time() - t0, 2)
        self.setup.update(getattr(self.gdet, 'setup_times', {}))
        self.setup['host_threads'] = _native_host_threads()
        log('rank %d: geometry on device in %.1fs (%.2f GB; %s)' % (rank, time.time() - t0,
                                                                   self.gdet.device_bytes() / 1e9, self.setup))
        self.nslots = args.nthreads_per_block * args.max_blocks
        self.rng = gpu.get_rng_states(self.nslots, seed=args.seed,
                                      first_subsequence=rng_first_subsequence(rank, self.nslots))
        self.photons = isotropic(nphotons, seed=PHOTON_SEED + rank)
        ph = self.photons
        self.pristine = SimpleNamespace(
            pos=ga.to_gpu(gpu.to_float3(ph.pos)), dir=ga.to_gpu(gpu.to_float3(ph.dir)),
            pol=ga.to_gpu(gpu.to_float3(ph.pol)), wavelengths=ga.to_gpu(ph.wavelengths),
            t=ga.to_gpu(ph.t), flags=ga.to_gpu(ph.flags), evidx=ga.to_gpu(ph.evidx), true_nphotons=nphotons)
        torch.cuda.synchronize()
        self.setup['setup_s'] = round(time.time() - t_setup, 2)
        self.counts = ga.zeros(self.gdet.nchannels, np.uint32)
        self.reduced = {}
        self.group = max(1, min(args.steps, args.pipeline_depth)) if args.pipeline else 1
        # the batches' device arrays, allocated once before any timing (a step
        # restores its batch from the device-resident source, D2D, inside the
        # timed region -- what GPUPhotons(pristine, ...) does, without the allocation)
        self.pool = [gpu.GPUPhotons(self.pristine, copy_flags=True, copy_triangles=False, copy_weights=False)
                     for _ in range(max(self.group, args.warmup, 2 if args.pipeline else 1))]

    def sync(self):
        self.torch.cuda.synchronize()

    def _restore(self, gp):
        for f in ('pos', 'dir', 'pol', 'wavelengths', 't', 'flags', 'evidx'):
            getattr(gp, f).tensor.copy_(getattr(self.pristine, f).tensor)
        gp.last_hit_triangles.fill(-1)
        gp.weights.fill(1.0)

    def prepare(self, m):
        """The next run(m)'s m input batches filled now (device copies of the
        source batch), so that run(m) starts from resident inputs."""
        for gp in self.pool[:m]:
            self._restore(gp)
        self.prepared = m

    def run(self, m, pipeline=None):
        """m steps: m fresh copies of the source batch propagated with one
        rng_states -- pipelined (gpu.propagate_batches: each batch's tail runs
        on a second stream while the next batch starts; results identical to m
        propagate calls) unless --no-pipeline -- then each batch's hit-channel
        reduce."""
        import ctypes
        from chroma import gpu
        from chroma.gpu import _native, shard
        from chroma.gpu.tools import current_stream
        args = self.args
        pipeline = args.pipeline if pipeline is None else pipeline
        gps = self.pool[:m]
        if getattr(self, 'prepared', 0) != m:
            for gp in gps:
                self._restore(gp)
        self.prepared = 0
        kw = dict(nthreads_per_block=args.nthreads_per_block, max_blocks=args.max_blocks, max_steps=args.max_steps)
        if pipeline and m > 1:
            sts = list(gpu.propagate_batches(gps, self.gdet, self.rng, **kw))
        else:
            sts = []
            for gp in gps:
                gp.propagate(self.gdet, self.rng, **kw)
                sts.append(gp.last_stats)
        for gp in gps:
            # hit-channel reduce: detected photons per PMT channel on each rank,
            # SUM-reduced over ranks (RCCL for N > 1)
            self.counts.fill(0)
            _native.call('chr_channel_hit_counts', ctypes.byref(gp._desc()), 0, self.nphotons, 0x4,
                         self.gdet.solid_id_map.gpudata, self.gdet.solid_id_to_channel_index_gpu.gpudata,
                         self.counts.gpudata, self.gdet.nchannels, current_stream())
            self.reduced['counts'] = shard.allreduce_channel_counts(self.counts.tensor)
        self.reduced['gp'] = gps[-1]
        return sts

    def run_sequential(self, m):
        return self.run(m, pipeline=False)

    def at_max_steps(self, nbatches):
        """Photons of each of the last call's batches that ran out of steps: their
        history holds none of the terminal bits (NO_HIT, BULK_ABSORB, SURFACE_DETECT,
        SURFACE_ABSORB, NAN_ABORT; propagate.cu:282-340 stops them alive at max_steps).
        Counted on the device from the output flags, after the timed region; None when
        the stats span more batches than the pool holds."""
        pool = getattr(self, 'pool', [])
        if nbatches == 0 or nbatches > len(pool):
            return [None] * nbatches
        dead = 0x1 | 0x2 | 0x4 | 0x8 | 0x8000
        return [int(((gp.flags.tensor & dead) == 0).sum().item()) for gp in pool[:nbatches]]

    def rank_report(self, stats):
        """This rank's own numbers from the timed steps' stats."""
        launch_ms = [float(s.trace_launch_ms[i]) for s in stats for i in range(s.trace_ms_n)]
        at_max = self.at_max_steps(len(stats))
        gp = self.reduced.get('gp')
        return {'rank': self.rank, 'photons_per_step': self.nphotons,
                'device': self.torch.cuda.get_device_properties(self.local).name, 'local_rank': self.local,
                'host': socket.gethostname(),
                'kernel_ms': sum(s.kernel_ms for s in stats), 'launches': sum(s.launches for s in stats),
                'host_steps': sum(s.steps_run for s in stats), 'host_syncs': sum(s.host_syncs for s in stats),
                'trace_ms': sum(s.trace_ms for s in stats), 'trace_launches': sum(s.trace_launches for s in stats),
                'trace_rays': sum(s.trace_rays for s in stats), 'launch_ms': launch_ms,
                'launch_rays': [int(stats[0].trace_launch_rays[i]) for i in range(stats[0].trace_ms_n)]
                if stats else [],
                'overflows': sum(s.stack_overflows for s in stats), 'flat': sum(s.flat_walks for s in stats),
                'flat_whole': sum(s.flat_walks_whole for s in stats),
                'detected_last_step': int(((gp.flags.get() & 4) != 0).sum()) if gp is not None else 0,
                'channel_hits_all_ranks': int(self.reduced['counts'].sum().item()) if 'counts' in self.reduced
                else 0,
                'setup': dict(self.setup, **host_memory()),
                'tail': [{'ms': round(s.tail_ms, 3), 'photons': int(s.tail_photons),
                          'max_steps': int(s.tail_max_steps), 'photons_at_max_steps': at_max[i],
                          'slowest_photon_ms': round(s.tail_max_cycles / 1e5, 3),
                          'slowest_photon_steps': int(s.tail_slowest_steps),
                          'long_photons': int(s.tail_long_photons),
                          'long_us_per_step': round(s.tail_long_ticks / 100.0 / max(1, s.tail_long_steps), 3),
                          'long_walk_us_per_step': round(s.tail_long_walk_ticks / 100.0 /
                                                         max(1, s.tail_long_steps), 3),
                          'long_walk_iterations_per_step': round(s.tail_long_walk_iterations /
                                                                 max(1, s.tail_long_steps), 2),
                          'long_paired_step_fraction': round(s.tail_long_paired_steps / max(1, s.tail_long_steps), 3)}
                         for i, s in enumerate(stats)]}

    def untimed_passes(self):
        """After timing: the counting variant (own-layout bytes, SIMD efficiency)
        and, with CHROMA_DEVICE_PROFILE=1, the device region profile."""
        from chroma.gpu import _native
        out = {}
        if not self.args.no_count:
            prev = os.environ.get('CHR_PROPAGATE_VARIANT')
            os.environ['CHR_PROPAGATE_VARIANT'] = '5'
            cst = self.run(1)[0]
            self.reduced.pop('gp', None)
            if prev is None:
                del os.environ['CHR_PROPAGATE_VARIANT']
            else:
                os.environ['CHR_PROPAGATE_VARIANT'] = prev
            self.sync()
            if cst.traversals:
                out['own_layout'] = {
                    'bytes_per_walk': (96.0 * cst.nodes_visited + 64.0 * cst.triangles_tested +
                                       52.0 * cst.traversals) / cst.traversals,
                    'nodes_per_photon': cst.nodes_visited / self.nphotons,
                    'triangles_per_photon': cst.triangles_tested / self.nphotons,
                    'traversals_per_photon': cst.traversals / self.nphotons,
                    'simd_efficiency_nodes': cst.nodes_visited / max(1.0, 64.0 * cst.wave_node_steps),
                    'simd_efficiency_triangles': cst.triangles_tested / max(1.0, 64.0 * cst.wave_triangle_steps),
                    'stack_overflows': int(cst.stack_overflows)}
        if _native.DEVICE_PROFILE:
            from chroma.gpu import profiler
            profiler.device_reset()
            self.run(1)
            self.reduced.pop('gp', None)
            self.sync()
            out['device_profile'] = {'regions': profiler.device_fetch(),
                                     'clock_khz': profiler.device_fetch.clock_khz,
                                     'library': os.path.basename(_native.library_path()),
                                     'cycles': 'lane-cycles of the shader clock (include/chroma_amd.h CHR_PROF_*)'}
        return out

    def device_info(self):
        from chroma.gpu import _native
        props = self.torch.cuda.get_device_properties(self.local)
        free_b, total_b = self.torch.cuda.mem_get_info(self.local)
        return {'device': {'name': props.name, 'arch': getattr(props, 'gcnArchName', ''),
                           'compute_units': props.multi_processor_count,
                           'hbm_total_gb': total_b / 1e9, 'hbm_free_gb_after': free_b / 1e9},
                'kernels': _kernel_info(_native)}

    def detector_info(self):
        return {'triangles': len(self.det.mesh.triangles), 'bvh_nodes': len(self.det.bvh.nodes),
                'channels': self.det.num_channels()}

    # ------------------------------------------------------------ oracle checks
    def _oracle_batches(self, n, threads, rank=None, inputs=None):
        """The oracle on rank `rank`'s first n photons (default: this rank's; another
        rank's come as `inputs`, the arrays its gpu_sample sent) as two batches in
        order (the RNG states carried from one to the next, as two propagate calls),
        from that rank's own RNG subsequences.  Returns (hosts, walk stats, seconds)."""
        sys.path.insert(0, os.path.join(ROOT, 'oracle'))
        import oracle
        from chroma.event import Photons
        from chroma.gpu.packing import PackedGeometry
        if not hasattr(self, '_packed'):
            self._packed = PackedGeometry(self.det)
        a = self.args
        rank = self.rank if rank is None else rank
        ph = self.photons if inputs is None else Photons(inputs['pos'], inputs['dir'], inputs['pol'],
                                                         inputs['wavelengths'])
        cuts = [0, n // 2, n]
        hosts = [oracle.HostPhotons(Photons(ph.pos[lo:hi], ph.dir[lo:hi], ph.pol[lo:hi], ph.wavelengths[lo:hi]))
                 for lo, hi in zip(cuts[:-1], cuts[1:])]
        st = oracle.rng_init(self.nslots, seed=a.seed, first_subsequence=rng_first_subsequence(rank, self.nslots))
        tot = {}
        t0 = time.time()
        for h in hosts:
            s = oracle.propagate(self._packed, h, st, self.nslots, a.nthreads_per_block, a.max_blocks, a.max_steps,
                                 threads=threads)
            for k, v in s.items():
                tot[k] = tot.get(k, 0) + v
        return hosts, tot, time.time() - t0

    def cpu_baseline(self, budget_s, threads):
        """Oracle (plain C port of the reference kernel, OpenMP) on a bounded
        sample of the same workload (grown until it takes ~budget/4 .. budget/2
        seconds); also returns the oracle's photons (the parity reference) and
        its walk counts on the reference BVH (roofline bytes).  --parity-photons
        fixes the sample instead (reproducible: the line records n either way)."""
        fixed = getattr(self.args, 'parity_photons', 0)
        n = min(self.nphotons, fixed) if fixed else 4000
        while True:
            hosts, stats, dt = self._oracle_batches(n, threads)
            if fixed or dt > budget_s / 4 or n * 4 > self.nphotons:
                break
            n = int(min(self.nphotons, n * max(2.0, min(8.0, (budget_s / 2) / max(dt, 1e-3)))))
        cpu = dict(value=n / dt, unit='photons/s', cores=threads, kind='port',
                   sample='%d of the same isotropic photons (two propagate calls of %d and %d, one RNG state set), '
                          'same geometry and launch shape, max_steps=%d; %.1fs on %d threads (nproc %d)' % (
                              n, n // 2, n - n // 2, self.args.max_steps, dt, threads, os.cpu_count() or 0))
        return cpu, stats, n, hosts

    PARITY_FIELDS = ('flags', 'last_hit_triangles', 'pos', 'dir', 'pol', 't', 'wavelengths')

    def gpu_sample(self, n, pipeline):
        """This rank's first n photons propagated on its GPU as two batches (same
        RNG initialisation and launch shape as the oracle's) -- through
        propagate_batches when the headline is pipelined, one propagate call each
        otherwise.  Returns the photons' fields (host arrays) and the run's facts:
        what a rank > 0 sends to rank 0, which runs the oracle for every rank."""
        from chroma import gpu
        from chroma.event import Photons
        a = self.args
        ph = self.photons
        cuts = [0, n // 2, n]
        gps = [gpu.GPUPhotons(Photons(ph.pos[lo:hi], ph.dir[lo:hi], ph.pol[lo:hi], ph.wavelengths[lo:hi]),
                              copy_flags=True, copy_triangles=False, copy_weights=False)
               for lo, hi in zip(cuts[:-1], cuts[1:])]
        rng = gpu.get_rng_states(self.nslots, seed=a.seed,
                                 first_subsequence=rng_first_subsequence(self.rank, self.nslots))
        kw = dict(nthreads_per_block=a.nthreads_per_block, max_blocks=a.max_blocks, max_steps=a.max_steps)
        if pipeline:
            sts = gpu.propagate_batches(gps, self.gdet, rng, **kw)
        else:
            sts = []
            for gp in gps:
                gp.propagate(self.gdet, rng, **kw)
                sts.append(gp.last_stats)
        got = [gp.get() for gp in gps]
        # the inputs go with the photons: rank 0 runs the oracle on them (regenerating
        # another rank's whole shard to take its first n photons would cost rank 0 the
        # memory of every shard)
        inputs = {f: np.ascontiguousarray(getattr(ph, f)[:n]) for f in ('pos', 'dir', 'pol', 'wavelengths')}
        return {'rank': self.rank, 'n': int(n), 'batches': [int(c) for c in np.diff(cuts)], 'inputs': inputs,
                'path': 'propagate_batches (pipelined)' if pipeline else 'propagate (sequential)',
                'stack_overflows': int(sum(s.stack_overflows for s in sts)),
                'photons': {f: np.concatenate([getattr(o, f) for o in got]) for f in self.PARITY_FIELDS}}

    def compare(self, sample, hosts):
        """Parity of a rank's GPU sample against the oracle's photons (hosts):
        flags, last-hit triangles and channels bit-exact, floats as max relative."""
        got = sample['photons']
        rank = sample['rank']
        solid_map = np.asarray(self.det.solid_id, np.int64)
        s2c = np.asarray(self.det.solid_id_to_channel_index, np.int64)

        def cat(objs, f):
            return np.concatenate([getattr(o, f) for o in objs])

        def channel(flags, last_hit):
            ch = np.full(len(flags), -1, np.int64)
            det = ((flags & 4) != 0) & (last_hit > -1)
            ch[det] = s2c[solid_map[last_hit[det]]]
            return ch

        def max_rel(x, y):
            x = np.asarray(x, np.float64)
            y = np.asarray(y, np.float64)
            return float(np.max(np.abs(x - y) / np.maximum(np.abs(y), 1e-30))) if x.size else 0.0

        n = sample['n']
        gf, hf = got['flags'], cat(hosts, 'flags')
        gl, hl = got['last_hit_triangles'], cat(hosts, 'last_hit_triangles')
        ch_gpu, ch_ref = channel(gf, gl), channel(hf, hl)
        rel = max(max_rel(got[f], cat(hosts, f)) for f in ('pos', 't', 'wavelengths'))
        dp = max(float(np.max(np.abs(got[f] - cat(hosts, f)))) if n else 0.0 for f in ('dir', 'pol'))
        floats = {f: float_contract(got[f], cat(hosts, f), f, sample['batches'], gf, hf, gl, hl)
                  for f in ('pos', 'dir', 'pol', 't', 'wavelengths')}
        out = {'rank': rank, 'n': int(n), 'batches': sample['batches'], 'path': sample['path'],
               'rng_first_subsequence': rng_first_subsequence(rank, self.nslots),
               'photon_seed': PHOTON_SEED + rank,
               'flags_equal': bool(np.array_equal(gf, hf)), 'last_hit_equal': bool(np.array_equal(gl, hl)),
               'channel_equal': bool(np.array_equal(ch_gpu, ch_ref)),
               'flags_mismatches': int(np.count_nonzero(gf != hf)),
               'last_hit_mismatches': int(np.count_nonzero(gl != hl)),
               'detected': int(np.count_nonzero(ch_ref >= 0)), 'max_rel': rel, 'dir_pol_max_abs': dp,
               'rule': PARITY_RULE, 'floats': floats,
               'bit_identical': bool(all(v['max_abs'] == 0.0 for v in floats.values())),
               'binned_first_step': bool(n // 2 >= (1 << 20)),
               'stack_overflows': sample['stack_overflows'], 'oracle_on_rank': self.rank}
        bad = np.flatnonzero((gf != hf) | (gl != hl))
        if bad.size:
            out['first_discrete_mismatches'] = [photon_record(i, sample['batches'], gf, hf, gl, hl) for i in bad[:8]]
        out['ok'] = bool(out['flags_equal'] and out['last_hit_equal'] and out['channel_equal'] and
                         all(v['violations'] == 0 for v in floats.values()))
        return out

    def check(self, full, budget_s, threads, sample):
        """Rank 0 (full): cpu_baseline + parity on the adaptive sample.  Otherwise
        parity on `sample` photons of this rank's shard, oracle run here.  Returns
        (cpu_baseline or None, oracle walk stats, parity)."""
        if full:
            cpu, stats, n, hosts = self.cpu_baseline(budget_s, threads)
        else:
            n = min(self.nphotons, sample)
            hosts, stats, _ = self._oracle_batches(n, threads)
            cpu = None
        return cpu, stats, self.compare(self.gpu_sample(n, self.args.pipeline), hosts)

    def check_rank(self, sample, threads):
        """On rank 0: the oracle for another rank's GPU sample (that rank's photon
        seed and RNG subsequences; only they differ, the geometry is rank 0's),
        compared photon by photon.  The other ranks build no host geometry copy."""
        hosts, _, _ = self._oracle_batches(sample['n'], threads, rank=sample['rank'], inputs=sample['inputs'])
        return self.compare(sample, hosts)


WORKLOAD = PropagateWorkload     # replaced by tests/bench_stub_main.py (CPU rehearsal of the rank logic)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument('--gpus', type=int, default=1,
                    help='GPUs (ranks); > 1 without WORLD_SIZE in the environment starts the ranks itself')
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--photons', type=int, default=10_000_000, help='photons per GPU per step (weak scaling)')
    ap.add_argument('--total-photons', type=int, default=0,
                    help='photons per step over all GPUs (strong scaling; overrides --photons)')
    ap.add_argument('--detector', default='29k', choices=sorted(DETECTORS))
    ap.add_argument('--max-steps', type=int, default=1000)
    ap.add_argument('--nthreads-per-block', type=int, default=512)
    ap.add_argument('--max-blocks', type=int, default=1024)
    ap.add_argument('--seed', type=int, default=1)
    ap.add_argument('--cpu-budget', type=float, default=20.0, help='seconds of CPU-baseline work')
    ap.add_argument('--parity-photons', type=int, default=0,
                    help='rank 0: a fixed parity / cpu_baseline sample of this many photons (0: grown to '
                         '~--cpu-budget/4 .. /2 seconds of oracle work; the line records the n used)')
    ap.add_argument('--no-preflight', action='store_true',
                    help='run even when the host-memory pre-flight says the local ranks do not fit')
    ap.add_argument('--allow-parity-failure', action='store_true',
                    help='exit 0 even when the parity check fails (diagnostic runs)')
    ap.add_argument('--rank-parity-photons', type=int, default=1 << 17,
                    help='photons of its own shard each rank > 0 checks against the oracle')
    ap.add_argument('--no-cpu-baseline', action='store_true', help='also skips the parity check')
    ap.add_argument('--no-count', action='store_true',
                    help='skip the untimed counting pass (profiling runs: keeps rocprof averages to one variant)')
    ap.add_argument('--no-pipeline', dest='pipeline', action='store_false',
                    help='one synchronous propagate per step (no tail / next-batch overlap)')
    ap.add_argument('--pipeline-depth', type=int, default=32,
                    help='steps per pipelined call (each holds its own copy of the batch in HBM)')
    ap.add_argument('--timing-steps', type=int, default=5,
                    help='untimed pipelined steps with every per-slot timing event recorded, after the timed '
                         'steps (detail.slot_timing_pass, detail.kernel_ms_per_step; 0: skip)')
    ap.add_argument('--sequential-steps', type=int, default=20,
                    help='after the pipelined headline: this many one-call-per-step steps, timed the same way '
                         '(detail.sequential; 0: skip)')
    ap.add_argument('--cache-dir', default=os.environ.get('CHROMA_BENCH_CACHE', '/tmp/chroma_bench_cache'))
    args = ap.parse_args(argv)
    if args.gpus < 1:
        ap.error('--gpus must be >= 1')
    if args.total_photons and args.total_photons < args.gpus:
        ap.error('--total-photons must give every GPU at least one photon')
    return args


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def spawn_ranks(n, cmd):
    """Start n rank processes of `cmd` (this script, same arguments) with the
    torchrun environment, one GPU each (LOCAL_RANK), and wait.  Called before
    this process touches any GPU.  A rank that fails ends the others; the exit
    status is the first failing rank's (0 when all succeed)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), GROUP_RANK='0')
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            c = p.poll()
            if c is None:
                continue
            alive.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                log('bench.py: rank %d exited with %d; stopping the other ranks' % (procs.index(p), c))
                for q in alive:
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def rank_env():
    return (int(os.environ.get('WORLD_SIZE', '1')), int(os.environ.get('RANK', '0')),
            int(os.environ.get('LOCAL_RANK', '0')))


def run_rank(args):
    world, rank, local = rank_env()
    if world != args.gpus:
        raise SystemExit('bench.py: --gpus %d but WORLD_SIZE=%d: the line would mislabel the run' % (args.gpus, world))
    import torch
    dist = None
    on_gpu = torch.cuda.is_available()
    if on_gpu:
        torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if on_gpu:
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group('gloo')
        if dist.get_world_size() != args.gpus:
            raise SystemExit('bench.py: process group has %d ranks, --gpus %d' % (dist.get_world_size(), args.gpus))
    nphotons = photons_for_rank(args, rank, world)
    # libchroma_amd's host-side builds use this rank's share of the job's cores
    # (the box's cgroup quota, not nproc), not a full team per rank
    local_world = int(os.environ.get('LOCAL_WORLD_SIZE', str(world)))
    preflight = preflight_host_memory(args.detector, local_world)
    if world > 1:
        # one decision for the whole job (local rank 0's view of the node), taken before
        # any rank allocates its geometry
        box = [preflight]
        dist.broadcast_object_list(box, src=0)
        preflight = box[0]
    if not preflight['fits'] and not args.no_preflight:
        raise SystemExit('bench.py: host memory pre-flight refused the run: %d local ranks of the %s detector need '
                         '~%.0f GB of host memory (rank 0 %.0f GB, each other rank %.0f GB) and %.0f GB is available '
                         '(--no-preflight to run anyway)' % (
                             local_world, args.detector, preflight['need_gb'], preflight['per_rank_gb']['rank0'],
                             preflight['per_rank_gb']['other'], preflight['available_gb']))
    from chroma.gpu import _native
    _native.set_host_threads(max(1, usable_cpus() // max(1, local_world)))
    wl = WORKLOAD(args, rank, world, local, dist, nphotons)

    # pipelined runs warm up with at least 2 steps: a 1-batch call does not use
    # (so would not allocate) the batches' extra buffer contexts, streams and events
    warmup = max(args.warmup, 2) if (args.pipeline and args.warmup > 0) else args.warmup
    elapsed, per_step, stats = timed_loop(wl.run, args.steps, warmup, dist, wl.sync, wl.group,
                                          getattr(wl, 'prepare', None))
    total_photons = nphotons * args.steps
    if dist is not None:
        total_photons = int(round(_allreduce(dist, float(total_photons), 'sum')))
    report = wl.rank_report(stats)
    seq = None
    if args.pipeline and args.sequential_steps > 0:
        # warm-up first: a propagate call uses its own buffer context, whose first use
        # allocates it (r03's 5-step figure, 350.7 M/s, timed that allocation)
        s_el, _, _ = timed_loop(wl.run_sequential, args.sequential_steps, 2, dist, wl.sync, 1)
        s_total = nphotons * args.sequential_steps
        if dist is not None:
            s_total = _allreduce(dist, float(s_total), 'sum')
        seq = {'photons_per_s': s_total / s_el, 'steps': args.sequential_steps, 'warmup': 2,
               'ms_per_step': 1e3 * s_el / args.sequential_steps,
               'path': 'one GPUPhotons.propagate call per step (the reference caller\'s loop)'}
    wl.reduced.pop('gp', None)
    # per-slot timing events (kernel time per step, tail launch times) cost ~0.6% of the
    # step when recorded (CHR_SLOT_TIMING): the timed steps record only the
    # trace launches' pair (the roofline's launch times); a short untimed pass with every
    # slot's events reports the rest
    timing_pass = None
    tsteps = min(args.timing_steps, len(getattr(wl, 'pool', [])) or args.timing_steps)
    if tsteps > 0:
        prev = os.environ.get('CHR_SLOT_TIMING')
        os.environ['CHR_SLOT_TIMING'] = '1'
        t_el, _, t_stats = timed_loop(wl.run, tsteps, 0, dist, wl.sync, min(wl.group, tsteps))
        t_rep = wl.rank_report(t_stats)
        wl.reduced.pop('gp', None)
        if prev is None:
            del os.environ['CHR_SLOT_TIMING']
        else:
            os.environ['CHR_SLOT_TIMING'] = prev
        timing_pass = {'steps': tsteps, 'ms_per_step': 1e3 * t_el / tsteps,
                       'kernel_ms_per_step': t_rep['kernel_ms'] / tsteps,
                       'trace_ms_per_step': t_rep['trace_ms'] / tsteps,
                       'tail_ms': [t['ms'] for t in t_rep['tail']],
                       'note': 'untimed pass after the timed steps with every slot event recorded '
                               '(CHR_SLOT_TIMING=1); the timed steps record only the trace launch pairs'}
    extra = wl.untimed_passes()

    # oracle checks: ranks > 0 propagate a sample of their own shard on their GPU and
    # send the photons to rank 0; rank 0 runs the timed cpu_baseline alone on the host
    # (its own parity), then the oracle for every other rank's sample -- only rank 0
    # holds a host copy of the geometry's packed tables (PackedGeometry)
    # this rank's memory before the oracle checks (rank 0's checks hold the oracle's
    # host copy of the geometry and every rank's sample: reported apart)
    report.update(host_memory())
    check, samples = None, None
    if not args.no_cpu_baseline:
        mine = None
        if rank > 0:
            mine = wl.gpu_sample(min(nphotons, args.rank_parity_photons), args.pipeline)
        if dist is not None:
            samples = [None] * world if rank == 0 else None
            dist.gather_object(mine, samples, dst=0)
        if rank == 0:
            check = wl.check(True, args.cpu_budget, usable_cpus(), 0)
            per_rank = [check[2]] + [wl.check_rank(smp, usable_cpus()) for smp in (samples or [None])[1:]]
            check = (check[0], check[1], check[2], per_rank)
    report['host_peak_rss_gb_after_checks'] = host_memory().get('host_peak_rss_gb')
    if dist is not None:
        reports = [None] * world
        dist.all_gather_object(reports, report)
    else:
        reports = [report]

    rc = 0
    if rank == 0:
        steps = max(1, args.steps)
        r0 = reports[0]
        detail = {'pipelined_steps_per_call': wl.group, 'warmup_steps_run': warmup, 'preflight': preflight,
                  # the timed steps' input batches were filled before t0 (timed_loop's prepare;
                  # bench.py since 40b6d98) rather than restored inside the timed region
                  'inputs_prefilled': getattr(wl, 'prepare', None) is not None and wl.group >= args.steps,
                  'ranks_seen': len(reports),
                  'ranks': [dict({k: rep[k] for k in ('rank', 'local_rank', 'host', 'device', 'photons_per_step')},
                                 setup=rep.get('setup'), host_rss_gb=rep.get('host_rss_gb'),
                                 host_peak_rss_gb=rep.get('host_peak_rss_gb'),
                                 host_peak_rss_gb_after_checks=rep.get('host_peak_rss_gb_after_checks'))
                            for rep in reports],
                  'kernel_ms_per_step': (timing_pass['kernel_ms_per_step'] if timing_pass else r0['kernel_ms'] / steps),
                  'trace_ms_per_step': r0['trace_ms'] / steps,
                  'launches_per_step': r0['launches'] / steps,
                  'host_steps_per_propagate': r0['host_steps'] / steps,
                  'stream_draining_host_syncs_per_propagate': r0['host_syncs'] / steps,
                  'stack_overflows': int(sum(r['overflows'] for r in reports)),
                  'flat_walks_trace': int(sum(r['flat'] for r in reports)),
                  'flat_walks_tail': int(sum(r['flat_whole'] for r in reports)),
                  'tail_launch': r0['tail'],
                  'first_propagate_trace_launches': [{'rays': r, 'ms': round(float(m), 3)} for r, m in
                                                     zip(r0['launch_rays'], r0['launch_ms'][:len(r0['launch_rays'])])],
                  'detected_fraction': r0['detected_last_step'] / max(1, nphotons),
                  'channel_hits_all_ranks': r0['channel_hits_all_ranks'],
                  'sequential': seq, 'slot_timing_pass': timing_pass}
        detail.update(wl.device_info())
        detail.update(extra)
        result = result_line(args, world, elapsed, per_step, total_photons, wl.detector_info(), detail)
        if check is not None:
            cpu, ostats, par, per_rank = check
            result['cpu_baseline'] = cpu
            nsample = par['n']
            detail['reference_bvh_nodes_per_photon'] = ostats['nodes_visited'] / nsample
            detail['reference_bvh_triangles_per_photon'] = ostats['tris_tested'] / nsample
            detail['bytes_per_photon_alg_8d'] = 120.0 + (16.0 * ostats['nodes_visited'] + 48.0 * ostats['tris_tested'] +
                                                         4.0 * ostats['traversals']) / nsample
            parity = dict(par)
            if world > 1:
                parity['per_rank'] = per_rank
                parity['all_ranks_equal'] = all(p is not None and p['flags_equal'] and p['last_hit_equal'] and
                                                p['channel_equal'] for p in parity['per_rank'])
            parity['ok'] = bool(par['ok'] and all(p is not None and p['ok'] for p in per_rank))
            result['parity'] = parity
            if r0['trace_launches']:
                result['roofline'] = roofline(args, reports, ostats)
        result['geometry_md5_match'] = geometry_md5_check(args.detector, getattr(wl, 'det', None), detail)
        print(json.dumps(result), flush=True)
        if check is not None and not result['parity']['ok']:
            log('bench.py: PARITY FAILED against the oracle (parity.ok false; parity.floats / '
                'first_discrete_mismatches name the photons)')
            rc = 0 if args.allow_parity_failure else 3
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return rc


def main(argv=None):
    args = parse_args(argv)
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        return spawn_ranks(args.gpus, [sys.executable, os.path.abspath(sys.argv[0])] +
                           (sys.argv[1:] if argv is None else list(argv)))
    return run_rank(args)


if __name__ == '__main__':
    sys.exit(main())
