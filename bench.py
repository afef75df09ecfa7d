#!/usr/bin/env python
"""Benchmark: propagated photons/s of GPUPhotons.propagate (the reference's
hot path, chroma/gpu/photon.py:226-293) on a demo PMT detector.

One "step" = one propagate of a fresh batch of isotropic photons (BASELINE.md
section 3 source: centre point source, seed 20260102) to termination or
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
random numbers).  detail.step_ms is then each call's time split over its steps.

Multi-GPU: one process per GPU (torchrun), geometry replicated, photons
sharded (each rank propagates its own batch: weak scaling, RNG subsequences
disjoint per rank).  Each step ends with the hit-channel reduce: detected
photons are histogrammed per PMT channel on the device and SUM-reduced over
the ranks (RCCL, chroma.gpu.shard) -- the only exchange the path has.  The
timed region is bracketed by barriers and the max over ranks is reported.

Parity: rank 0 runs the CPU oracle (cpu_baseline leg, the only place bench.py
touches oracle/) on a bounded sample of the same photons with the same RNG
initialisation, then propagates the SAME sample on the GPU and compares the
two photon by photon (history flags, last-hit triangles and channels
bit-exact; positions, directions, polarisations, times and wavelengths as a
max relative difference) -- every bench line checks its own workload.

Roofline: the dominant kernel is trace_kernel, the
BVH walk of every one-step launch.  It is bound by HBM/L2 latency-bandwidth on
dependent node/triangle gathers.
    achieved = algorithmic bytes per trace launch / average trace launch time
with the average from HIP events around each trace launch on its stream, and
the algorithmic bytes of section 8(d): per walk 16 * reference-BVH nodes +
48 * reference triangles + 4, counted by the CPU oracle walking the REFERENCE
BVH in the reference's DFS order on the cpu_baseline sample of the same
workload, times the rays of the launch.  traffic = HBM bytes per trace launch
from the rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this workload; those
counters cannot be read from inside this process, so the value is copied
from the committed PMC summary (profiles/latest_pmc.json) and labelled so.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))

import numpy as np  # noqa: E402

METRIC = 'propagated photons/sec, 29k-PMT detector, 10M isotropic photons, 1/2/4/8 GPUs'
HBM_PEAK_GBS = 8000.0
PHOTON_SEED = 20260102


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
    the node-local cache; the other ranks wait at a barrier, then load it."""
    if dist is None or not cache_dir:
        return build_geometry(name, cache_dir)
    if rank == 0:
        det = build_geometry(name, cache_dir)
    dist.barrier()
    if rank != 0:
        det = build_geometry(name, cache_dir)
    return det


def rng_first_subsequence(rank, nslots):
    """Rank r's RNG slots are curand subsequences [r*nslots, (r+1)*nslots):
    disjoint streams, and rank 0 draws what a single-GPU run draws."""
    return rank * nslots


def timed_loop(run, steps, warmup, dist, sync, group=1):
    """W untimed steps, then K timed steps bracketed by barrier + sync on both
    sides; run(m) performs m steps and returns their results (m > 1: one
    pipelined call, see main).  Returns (elapsed max over ranks, this rank's
    per-step seconds -- a group's time split evenly over its steps --, per-step
    results)."""
    if warmup:
        run(warmup)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    marks, results, per_step = [], [], []
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
        import torch
        dev = 'cuda' if (torch.cuda.is_available() and dist.get_backend() != 'gloo') else 'cpu'
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed, per_step, results


def result_line(args, world, elapsed, per_step_s, detector_info, detail):
    total = args.photons * world * args.steps
    value = total / elapsed
    return {
        'metric': METRIC, 'value': value, 'unit': 'photons/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': 1e3 * elapsed / args.steps, 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': (value / 2.5e6) if args.detector == '29k' else None,
        'dtype': 'f32', 'data': 'synthetic isotropic point source (BASELINE.md section 3), seed %d+rank' % PHOTON_SEED,
        'config': dict({'workload': 'GPUPhotons.propagate of %d isotropic photons per GPU per step on %s, '
                                    'max_steps=%d, launch shape %dx%d (%d RNG slots)' % (
                                        args.photons, DETECTORS[args.detector][0], args.max_steps,
                                        args.nthreads_per_block, args.max_blocks,
                                        args.nthreads_per_block * args.max_blocks),
                        'detector': args.detector, 'photons_per_gpu': args.photons, 'max_steps': args.max_steps,
                        'parallelism': 'photon-sharded x%d, geometry replicated' % world}, **detector_info),
        'detail': dict({'step_ms': [round(1e3 * s, 3) for s in per_step_s]}, **detail),
        'roofline': None, 'cpu_baseline': None, 'parity': None,
    }


def cpu_baseline(packed, photons, nslots, ntpb, max_blocks, max_steps, seed, budget_s, threads):
    """Oracle (plain C port of the reference kernel, OpenMP) on a bounded
    sample of the same workload; also returns the oracle's photons (the parity
    reference) and its walk counts on the reference BVH (roofline bytes)."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    from chroma.event import Photons
    n = 2000
    while True:
        sample = Photons(photons.pos[:n], photons.dir[:n], photons.pol[:n], photons.wavelengths[:n])
        host = oracle.HostPhotons(sample)
        st = oracle.rng_init(nslots, seed=seed)
        t0 = time.time()
        stats = oracle.propagate(packed, host, st, nslots, ntpb, max_blocks, max_steps, threads=threads)
        dt = time.time() - t0
        if dt > budget_s / 4 or n * 4 > len(photons.pos):
            break
        n = int(min(len(photons.pos), n * max(2.0, min(8.0, (budget_s / 2) / max(dt, 1e-3)))))
    b_alg = 120.0 + (16.0 * stats['nodes_visited'] + 48.0 * stats['tris_tested'] + 4.0 * stats['traversals']) / n
    cpu = dict(value=n / dt, unit='photons/s', cores=threads, kind='port',
               sample='%d of the same isotropic photons, same geometry and launch shape, max_steps=%d; %.1fs on %d '
                      'threads (nproc %d)' % (n, max_steps, dt, threads, os.cpu_count() or 0))
    return cpu, b_alg, stats, n, host


def gpu_parity(gdet, photons, n, host, args, solid_map, s2c):
    """Propagate the oracle's sample on the GPU (same RNG initialisation, same
    launch shape) and compare photon by photon."""
    from chroma import gpu
    from chroma.event import Photons
    sample = Photons(photons.pos[:n], photons.dir[:n], photons.pol[:n], photons.wavelengths[:n])
    nslots = args.nthreads_per_block * args.max_blocks
    gp = gpu.GPUPhotons(sample, copy_flags=True, copy_triangles=False, copy_weights=False)
    gp.propagate(gdet, gpu.get_rng_states(nslots, seed=args.seed), nthreads_per_block=args.nthreads_per_block,
                 max_blocks=args.max_blocks, max_steps=args.max_steps)
    got = gp.get()

    def channel(flags, last_hit):
        ch = np.full(len(flags), -1, np.int64)
        det = ((flags & 4) != 0) & (last_hit > -1)
        ch[det] = s2c[solid_map[last_hit[det]]]
        return ch

    def max_rel(a, b):
        a = np.asarray(a, np.float64)
        b = np.asarray(b, np.float64)
        return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30))) if a.size else 0.0

    flags_eq = bool(np.array_equal(got.flags, host.flags))
    hits_eq = bool(np.array_equal(got.last_hit_triangles, host.last_hit_triangles))
    ch_gpu, ch_ref = channel(got.flags, got.last_hit_triangles), channel(host.flags, host.last_hit_triangles)
    rel = max(max_rel(got.pos, host.pos), max_rel(got.t, host.t), max_rel(got.wavelengths, host.wavelengths))
    dp = max(float(np.max(np.abs(got.dir - host.dir))) if n else 0.0,
             float(np.max(np.abs(got.pol - host.pol))) if n else 0.0)
    return {'n': int(n), 'flags_equal': flags_eq, 'last_hit_equal': hits_eq,
            'channel_equal': bool(np.array_equal(ch_gpu, ch_ref)),
            'flags_mismatches': int(np.count_nonzero(got.flags != host.flags)),
            'detected': int(np.count_nonzero(ch_ref >= 0)), 'max_rel': rel, 'dir_pol_max_abs': dp,
            'binned_first_step': bool(n >= (1 << 20)),
            'stack_overflows': int(gp.last_stats.stack_overflows)}


def _kernel_info(native):
    try:
        return native.kernel_info()
    except (AttributeError, native.NativeError) as e:     # an older library (A/B runs)
        return 'unavailable: %s' % e


def roofline(args, trace_ms, trace_launches, trace_rays, ref, launch_ms):
    """roofline object of the bench line for the dominant kernel (trace_kernel)."""
    launches = max(1, trace_launches)
    rays_per_launch = trace_rays / launches
    avg_launch_s = trace_ms / launches / 1e3
    per_walk = (16.0 * ref['nodes_visited'] + 48.0 * ref['tris_tested']) / ref['traversals'] + 4.0
    alg_per_launch = rays_per_launch * per_walk
    achieved = alg_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    lm = np.asarray(launch_ms, np.float64)
    rl = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
          'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
          'kernel': 'chr::trace_kernel (BVH walk of the one-step launches)',
          'basis': 'SURVEY 8(d): 16 B x reference-BVH nodes + 48 B x triangles + 4 B per walk '
                   '(oracle, reference DFS order, on the cpu_baseline sample)',
          'alg_bytes_per_launch': alg_per_launch, 'alg_bytes_per_walk': per_walk,
          'rays_per_launch': rays_per_launch, 'avg_launch_ms': 1e3 * avg_launch_s,
          'launches_timed': trace_launches,
          'launch_ms_min': float(lm.min()) if lm.size else None,
          'launch_ms_median': float(np.median(lm)) if lm.size else None,
          'launch_ms_max': float(lm.max()) if lm.size else None,
          'reference_bvh_nodes_per_walk': ref['nodes_visited'] / ref['traversals'],
          'reference_bvh_triangles_per_walk': ref['tris_tested'] / ref['traversals']}
    pmc_path = os.path.join(ROOT, 'profiles', 'latest_pmc.json')
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        w = pmc.get('workload', {})
        if (w.get('detector'), w.get('photons'), w.get('max_steps')) == (args.detector, args.photons, args.max_steps) \
                and pmc.get('kernel') == 'chr::trace_kernel' and 'hbm_bytes_per_launch' in pmc:
            rl['traffic'] = pmc['hbm_bytes_per_launch']
            rl['traffic_unit'] = 'bytes/launch (FETCH_SIZE x2 + WRITE_SIZE)'
            rl['traffic_source'] = 'copied, not measured in this run: %s (%s)' % (
                os.path.relpath(pmc_path, ROOT), pmc.get('source'))
    return rl


def main():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--photons', type=int, default=10_000_000, help='photons per GPU per step')
    ap.add_argument('--detector', default='29k', choices=sorted(DETECTORS))
    ap.add_argument('--max-steps', type=int, default=1000)
    ap.add_argument('--nthreads-per-block', type=int, default=512)
    ap.add_argument('--max-blocks', type=int, default=1024)
    ap.add_argument('--seed', type=int, default=1)
    ap.add_argument('--cpu-budget', type=float, default=20.0, help='seconds of CPU-baseline work')
    ap.add_argument('--no-cpu-baseline', action='store_true', help='also skips the parity check')
    ap.add_argument('--no-count', action='store_true',
                    help='skip the untimed counting pass (profiling runs: keeps rocprof averages to one variant)')
    ap.add_argument('--no-pipeline', dest='pipeline', action='store_false',
                    help='one synchronous propagate per step (no tail / next-batch overlap)')
    ap.add_argument('--pipeline-depth', type=int, default=32,
                    help='steps per pipelined call (each holds its own copy of the batch in HBM)')
    ap.add_argument('--cache-dir', default=os.environ.get('CHROMA_BENCH_CACHE', '/tmp/chroma_bench_cache'))
    args = ap.parse_args()

    import torch
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    from chroma import gpu
    from chroma.gpu import gpuarray as ga
    from chroma.gpu.packing import PackedGeometry
    from chroma.photon_source import isotropic
    from types import SimpleNamespace

    det = shared_geometry(args.detector, args.cache_dir, rank, dist)
    t0 = time.time()
    gdet = gpu.GPUDetector(det)
    log('rank %d: geometry on device in %.1fs (%.2f GB)' % (rank, time.time() - t0, gdet.device_bytes() / 1e9))
    nslots = args.nthreads_per_block * args.max_blocks
    rng = gpu.get_rng_states(nslots, seed=args.seed, first_subsequence=rng_first_subsequence(rank, nslots))

    photons = isotropic(args.photons, seed=PHOTON_SEED + rank)
    pristine = SimpleNamespace(
        pos=ga.to_gpu(gpu.to_float3(photons.pos)), dir=ga.to_gpu(gpu.to_float3(photons.dir)),
        pol=ga.to_gpu(gpu.to_float3(photons.pol)), wavelengths=ga.to_gpu(photons.wavelengths),
        t=ga.to_gpu(photons.t), flags=ga.to_gpu(photons.flags), evidx=ga.to_gpu(photons.evidx),
        true_nphotons=args.photons)
    torch.cuda.synchronize()

    import ctypes
    from chroma.gpu import _native, shard
    from chroma.gpu.tools import current_stream
    counts = ga.zeros(gdet.nchannels, np.uint32)
    reduced = {}

    group = max(1, min(args.steps, args.pipeline_depth)) if args.pipeline else 1
    # the batches' device arrays, allocated once before any timing (a step
    # restores its batch from the device-resident source, D2D, inside the timed
    # region -- what GPUPhotons(pristine, ...) does, without the allocation)
    pool = [gpu.GPUPhotons(pristine, copy_flags=True, copy_triangles=False, copy_weights=False)
            for _ in range(max(group, args.warmup, 2 if args.pipeline else 1))]

    def restore(gp):
        for f in ('pos', 'dir', 'pol', 'wavelengths', 't', 'flags', 'evidx'):
            getattr(gp, f).tensor.copy_(getattr(pristine, f).tensor)
        gp.last_hit_triangles.fill(-1)
        gp.weights.fill(1.0)

    def run(m):
        """m steps: m fresh copies of the source batch propagated with one
        rng_states -- pipelined (gpu.propagate_batches: each batch's tail runs
        on a second stream while the next batch starts; results identical to m
        propagate calls) unless --no-pipeline -- then each batch's hit-channel
        reduce."""
        gps = pool[:m]
        for gp in gps:
            restore(gp)
        kw = dict(nthreads_per_block=args.nthreads_per_block, max_blocks=args.max_blocks, max_steps=args.max_steps)
        if args.pipeline and m > 1:
            sts = list(gpu.propagate_batches(gps, gdet, rng, **kw))
        else:
            sts = []
            for gp in gps:
                gp.propagate(gdet, rng, **kw)
                sts.append(gp.last_stats)
        for gp in gps:
            # hit-channel reduce: detected photons per PMT channel on each rank,
            # SUM-reduced over ranks (RCCL for N > 1)
            counts.fill(0)
            _native.call('chr_channel_hit_counts', ctypes.byref(gp._desc()), 0, args.photons, 0x4,
                         gdet.solid_id_map.gpudata, gdet.solid_id_to_channel_index_gpu.gpudata, counts.gpudata,
                         gdet.nchannels, current_stream())
            reduced['counts'] = shard.allreduce_channel_counts(counts.tensor)
        reduced['gp'] = gps[-1]
        return sts

    # pipelined runs warm up with at least 2 steps: a 1-batch call does not use
    # (so would not allocate) the batches' extra buffer contexts, streams and events
    warmup = max(args.warmup, 2) if (args.pipeline and args.warmup > 0) else args.warmup
    elapsed, per_step, stats = timed_loop(run, args.steps, warmup, dist, torch.cuda.synchronize, group)
    gp = reduced.pop('gp')
    detected = int(((gp.flags.get() & 4) != 0).sum())
    del gp
    channel_hits = int(reduced['counts'].sum().item())     # all ranks, detected with a channel
    launch_ms = [s.trace_launch_ms[i] for s in stats for i in range(s.trace_ms_n)]
    launch_rays = [int(stats[0].trace_launch_rays[i]) for i in range(stats[0].trace_ms_n)] if stats else []
    live = dict(kernel_ms=sum(s.kernel_ms for s in stats), launches=sum(s.launches for s in stats),
                host_steps=sum(s.steps_run for s in stats), host_syncs=sum(s.host_syncs for s in stats),
                trace_ms=sum(s.trace_ms for s in stats),
                trace_launches=sum(s.trace_launches for s in stats), trace_rays=sum(s.trace_rays for s in stats),
                overflows=sum(s.stack_overflows for s in stats), flat=sum(s.flat_walks for s in stats),
                flat_whole=sum(s.flat_walks_whole for s in stats),
                tail=[{'ms': round(s.tail_ms, 3), 'photons': int(s.tail_photons), 'max_steps': int(s.tail_max_steps),
                       'slowest_photon_ms': round(s.tail_max_cycles / 1e5, 3),
                       'slowest_photon_steps': int(s.tail_slowest_steps),
                       'long_photons': int(s.tail_long_photons),
                       'long_us_per_step': round(s.tail_long_ticks / 100.0 / max(1, s.tail_long_steps), 3),
                       'long_walk_us_per_step': round(s.tail_long_walk_ticks / 100.0 / max(1, s.tail_long_steps), 3),
                       'long_walk_iterations_per_step': round(s.tail_long_walk_iterations / max(1, s.tail_long_steps),
                                                              2)} for s in stats])
    # untimed: same propagate with the counting kernel variant -> own-layout bytes and SIMD efficiency
    cst = None
    if not args.no_count:
        prev = os.environ.get('CHR_PROPAGATE_VARIANT')
        os.environ['CHR_PROPAGATE_VARIANT'] = '5'
        cst = run(1)[0]
        reduced.pop('gp', None)
        if prev is None:
            del os.environ['CHR_PROPAGATE_VARIANT']
        else:
            os.environ['CHR_PROPAGATE_VARIANT'] = prev
        torch.cuda.synchronize()

    # untimed, CHROMA_DEVICE_PROFILE=1 only (libchroma_amd_prof.so, whose timed numbers
    # carry the counters): the device region profile of one more propagate
    dprof = None
    if _native.DEVICE_PROFILE:
        from chroma.gpu import profiler
        profiler.device_reset()
        run(1)
        reduced.pop('gp', None)
        torch.cuda.synchronize()
        dprof = {'regions': profiler.device_fetch(), 'clock_khz': profiler.device_fetch.clock_khz,
                 'library': os.path.basename(_native.library_path()),
                 'cycles': 'lane-cycles of the shader clock (include/chroma_amd.h CHR_PROF_*)'}

    if rank == 0:
        props = torch.cuda.get_device_properties(local)
        free_b, total_b = torch.cuda.mem_get_info(local)
        steps = max(1, args.steps)
        detail = {'pipelined_steps_per_call': group, 'warmup_steps_run': warmup,
                  'kernel_ms_per_step': live['kernel_ms'] / steps,
                  'trace_ms_per_step': live['trace_ms'] / steps,
                  'launches_per_step': live['launches'] / steps,
                  'host_steps_per_propagate': live['host_steps'] / steps,
                  'stream_draining_host_syncs_per_propagate': live['host_syncs'] / steps,
                  'stack_overflows': int(live['overflows']),
                  'flat_walks_decomposed': int(live['flat']), 'flat_walks_whole': int(live['flat_whole']),
                  'tail_launch': live['tail'],
                  'first_propagate_trace_launches': [{'rays': r, 'ms': round(float(m), 3)} for r, m in
                                                     zip(launch_rays, launch_ms[:len(launch_rays)])],
                  'detected_fraction': detected / args.photons,
                  'channel_hits_all_ranks': channel_hits,
                  'device': {'name': props.name, 'arch': getattr(props, 'gcnArchName', ''),
                             'compute_units': props.multi_processor_count,
                             'hbm_total_gb': total_b / 1e9, 'hbm_free_gb_after': free_b / 1e9},
                  'kernels': _kernel_info(_native)}
        if dprof is not None:
            detail['device_profile'] = dprof
        if cst is not None and cst.traversals:
            detail['own_layout'] = {
                'bytes_per_walk': (96.0 * cst.nodes_visited + 64.0 * cst.triangles_tested + 52.0 * cst.traversals)
                / cst.traversals,
                'nodes_per_photon': cst.nodes_visited / args.photons,
                'triangles_per_photon': cst.triangles_tested / args.photons,
                'traversals_per_photon': cst.traversals / args.photons,
                'simd_efficiency_nodes': cst.nodes_visited / max(1.0, 64.0 * cst.wave_node_steps),
                'simd_efficiency_triangles': cst.triangles_tested / max(1.0, 64.0 * cst.wave_triangle_steps),
                'stack_overflows': int(cst.stack_overflows)}
        info = {'triangles': len(det.mesh.triangles), 'bvh_nodes': len(det.bvh.nodes),
                'channels': det.num_channels()}
        result = result_line(args, world, elapsed, per_step, info, detail)
        if not args.no_cpu_baseline and world == 1:
            threads = usable_cpus()
            packed = PackedGeometry(det)
            cpu, b_ref, ostats, nsample, host = cpu_baseline(packed, photons, nslots, args.nthreads_per_block,
                                                             args.max_blocks, args.max_steps, args.seed,
                                                             args.cpu_budget, threads)
            result['cpu_baseline'] = cpu
            detail['reference_bvh_nodes_per_photon'] = ostats['nodes_visited'] / nsample
            detail['reference_bvh_triangles_per_photon'] = ostats['tris_tested'] / nsample
            detail['bytes_per_photon_alg_8d'] = b_ref
            result['parity'] = gpu_parity(gdet, photons, nsample, host, args,
                                          np.asarray(det.solid_id, np.int64),
                                          np.asarray(det.solid_id_to_channel_index, np.int64))
            if live['trace_launches']:
                result['roofline'] = roofline(args, live['trace_ms'], live['trace_launches'], live['trace_rays'],
                                              ostats, launch_ms)
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
