#!/usr/bin/env python
"""Benchmark: propagated photons/s of GPUPhotons.propagate (the reference's
hot path, chroma/gpu/photon.py:226-293) on a demo PMT detector.

One "step" = one propagate of a fresh batch of isotropic photons (BASELINE.md
section 3 source: centre point source, seed 20260102) to termination or
max_steps (default 1000, the Simulation.simulate default), launch shape of
Simulation (nthreads_per_block=512, max_blocks=1024 -> 524,288 RNG slots).
Photon inputs are resident in HBM before the timed region; each step restores
them from a device-resident copy (D2D, inside the timed region).

Multi-GPU: one process per GPU (torchrun), geometry replicated, photons
sharded (each rank propagates its own batch: weak scaling, RNG subsequences
disjoint per rank).  Each step ends with the hit-channel reduce: detected
photons are histogrammed per PMT channel on the device and SUM-reduced over
the ranks (RCCL, chroma.gpu.shard) -- the only exchange the path has.  The
timed region is bracketed by barriers and the max over ranks is reported.

Roofline: the dominant kernel is trace_kernel, the
BVH walk of every one-step launch (the last, multi-step launch of the
reference's nsteps policy runs the fused step kernel).  It is bound by HBM/L2
latency-bandwidth on dependent node/triangle gathers.
    achieved = algorithmic bytes per trace launch / average trace launch time
with the average from HIP events around each trace launch on its stream, and
the algorithmic bytes of section 8(d): per walk 16 * reference-BVH nodes +
48 * reference triangles + 4, counted by the CPU oracle walking the REFERENCE
BVH in the reference's DFS order on the cpu_baseline sample of the same
workload (layout-independent, comparable across builds), times the rays of
the launch.  The bytes of this build's own layout (96-byte wide nodes, 64-byte
triangle records) are counted on every photon by one extra, untimed propagate
with the counting variant (CHR_PROPAGATE_VARIANT=5) and reported beside it;
traffic = HBM bytes per trace launch from the rocprofv3 FETCH_SIZE/WRITE_SIZE
passes of this workload (profiles/latest_pmc.json).
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


def cpu_baseline(packed, photons, nslots, ntpb, max_blocks, max_steps, seed, budget_s, threads):
    """Oracle (plain C port of the reference kernel, OpenMP) on a bounded
    sample of the same workload; also returns the per-photon algorithmic
    byte count for the roofline."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    from chroma.event import Photons
    n = 2000
    total_t = 0.0
    agg = None
    while True:
        sample = Photons(photons.pos[:n], photons.dir[:n], photons.pol[:n], photons.wavelengths[:n])
        host = oracle.HostPhotons(sample)
        st = oracle.rng_init(nslots, seed=seed)
        t0 = time.time()
        stats = oracle.propagate(packed, host, st, nslots, ntpb, max_blocks, max_steps, threads=threads)
        dt = time.time() - t0
        total_t, agg = dt, (n, stats)
        if dt > budget_s / 4 or n * 4 > len(photons.pos):
            break
        n = int(min(len(photons.pos), n * max(2.0, min(8.0, (budget_s / 2) / max(dt, 1e-3)))))
    n, stats = agg
    b_alg = 120.0 + (16.0 * stats['nodes_visited'] + 48.0 * stats['tris_tested'] + 4.0 * stats['traversals']) / n
    return dict(value=n / total_t, unit='photons/s', cores=threads, kind='port',
                sample='%d of the same isotropic photons, same geometry and launch shape, max_steps=%d; %.1fs on %d '
                       'threads' % (n, max_steps, total_t, threads)), b_alg, stats, n


def roofline(args, live, cst, ref, n):
    """roofline object of the bench line for the dominant kernel (trace_kernel).
    live: timed-region sums of the propagate stats; cst: counting pass (own
    layout); ref: oracle counts on the reference BVH (None without cpu_baseline)."""
    launches = max(1, live['trace_launches'])
    rays_per_launch = live['trace_rays'] / launches
    avg_launch_s = live['trace_ms'] / launches / 1e3
    own = None
    if cst is not None and cst.traversals:
        own = (96.0 * cst.nodes_visited + 64.0 * cst.triangles_tested + 52.0 * cst.traversals) / cst.traversals
    if ref is not None:
        per_walk, basis = (16.0 * ref['nodes_visited'] + 48.0 * ref['tris_tested']) / ref['traversals'] + 4.0, \
            'SURVEY 8(d): 16 B x reference-BVH nodes + 48 B x triangles + 4 B per walk (oracle, reference DFS order)'
    else:
        per_walk, basis = own, 'own layout: 96 B x wide nodes + 64 B x triangle records + 52 B per walk'
    alg_per_launch = rays_per_launch * per_walk if per_walk else 0.0
    achieved = alg_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    rl = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
          'frac': achieved / HBM_PEAK_GBS, 'traffic': None,
          'kernel': 'chr::trace_kernel (BVH walk of the one-step launches)',
          'basis': basis,
          'alg_bytes_per_launch': alg_per_launch,
          'alg_bytes_per_walk': per_walk,
          'rays_per_launch': rays_per_launch,
          'avg_launch_ms': 1e3 * avg_launch_s,
          'launches_timed': live['trace_launches']}
    if own is not None:
        rl['own_layout_bytes_per_walk'] = own
        rl['own_layout_achieved'] = rays_per_launch * own / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
        rl['nodes_per_photon'] = cst.nodes_visited / n
        rl['triangles_per_photon'] = cst.triangles_tested / n
        rl['traversals_per_photon'] = cst.traversals / n
        rl['simd_efficiency_nodes'] = cst.nodes_visited / max(1.0, 64.0 * cst.wave_node_steps)
        rl['simd_efficiency_triangles'] = cst.triangles_tested / max(1.0, 64.0 * cst.wave_triangle_steps)
    if ref is not None:
        rl['reference_bvh_nodes_per_walk'] = ref['nodes_visited'] / ref['traversals']
        rl['reference_bvh_triangles_per_walk'] = ref['tris_tested'] / ref['traversals']
    # HBM bytes per launch from the PMC passes (tools/rocprof_bench.sh) of this same workload
    pmc_path = os.path.join(ROOT, 'profiles', 'latest_pmc.json')
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        w = pmc.get('workload', {})
        if (w.get('detector'), w.get('photons'), w.get('max_steps')) == (args.detector, args.photons, args.max_steps) \
                and pmc.get('kernel') == 'chr::trace_kernel' and 'hbm_bytes_per_launch' in pmc:
            rl['traffic'] = pmc['hbm_bytes_per_launch']
            rl['traffic_unit'] = 'bytes/launch (FETCH_SIZE x2 + WRITE_SIZE)'
            rl['traffic_source'] = pmc.get('source')
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
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-count', action='store_true',
                    help='skip the untimed counting pass (profiling runs: keeps rocprof averages to one variant)')
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

    if dist is not None and args.cache_dir:
        # rank 0 builds (flatten + BVH, minutes for the 29k detector) and fills the
        # local cache; the other ranks of the node wait, then load it
        if rank == 0:
            det = build_geometry(args.detector, args.cache_dir)
        dist.barrier()
        if rank != 0:
            det = build_geometry(args.detector, args.cache_dir)
    else:
        det = build_geometry(args.detector, args.cache_dir)
    t0 = time.time()
    gdet = gpu.GPUDetector(det)
    log('rank %d: geometry on device in %.1fs (%.2f GB)' % (rank, time.time() - t0, gdet.device_bytes() / 1e9))
    nslots = args.nthreads_per_block * args.max_blocks
    rng = gpu.get_rng_states(nslots, seed=args.seed, first_subsequence=rank * nslots)

    photons = isotropic(args.photons, seed=20260102 + rank)
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

    def step():
        gp = gpu.GPUPhotons(pristine, copy_flags=True, copy_triangles=False, copy_weights=False)
        gp.propagate(gdet, rng, nthreads_per_block=args.nthreads_per_block, max_blocks=args.max_blocks,
                     max_steps=args.max_steps)
        # hit-channel reduce: detected photons per PMT channel on each rank,
        # SUM-reduced over ranks (RCCL for N > 1)
        counts.fill(0)
        _native.call('chr_channel_hit_counts', ctypes.byref(gp._desc()), 0, args.photons, 0x4,
                     gdet.solid_id_map.gpudata, gdet.solid_id_to_channel_index_gpu.gpudata, counts.gpudata,
                     gdet.nchannels, current_stream())
        reduced['counts'] = shard.allreduce_channel_counts(counts.tensor)
        return gp

    for _ in range(args.warmup):
        gp = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    live = dict(kernel_ms=0.0, launches=0, host_steps=0, trace_ms=0.0, trace_launches=0, trace_rays=0)
    for _ in range(args.steps):
        gp = step()
        ls = gp.last_stats
        live['kernel_ms'] += ls.kernel_ms
        live['launches'] += ls.launches
        live['host_steps'] += ls.steps_run
        live['trace_ms'] += ls.trace_ms
        live['trace_launches'] += ls.trace_launches
        live['trace_rays'] += ls.trace_rays
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device='cuda')
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    detected = int(((gp.flags.get() & 4) != 0).sum())
    channel_hits = int(reduced['counts'].sum().item())     # all ranks, detected with a channel
    # untimed: same propagate with the counting kernel variant -> algorithmic bytes
    cst = None
    if not args.no_count:
        prev = os.environ.get('CHR_PROPAGATE_VARIANT')
        os.environ['CHR_PROPAGATE_VARIANT'] = '5'
        cst = step().last_stats
        if prev is None:
            del os.environ['CHR_PROPAGATE_VARIANT']
        else:
            os.environ['CHR_PROPAGATE_VARIANT'] = prev
        torch.cuda.synchronize()

    if rank == 0:
        total = args.photons * world * args.steps
        value = total / elapsed
        result = {
            'metric': METRIC, 'value': value, 'unit': 'photons/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': 1e3 * elapsed / args.steps, 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': (value / 2.5e6) if args.detector == '29k' else None,
            'dtype': 'f32', 'data': 'synthetic isotropic point source (BASELINE.md section 3), seed 20260102+rank',
            'config': {'workload': 'GPUPhotons.propagate of %d isotropic photons per GPU per step on %s, '
                                   'max_steps=%d, launch shape %dx%d (524,288 RNG slots)' % (
                                       args.photons, DETECTORS[args.detector][0], args.max_steps,
                                       args.nthreads_per_block, args.max_blocks),
                       'detector': args.detector, 'photons_per_gpu': args.photons, 'max_steps': args.max_steps, 'triangles': len(det.mesh.triangles),
                       'bvh_nodes': len(det.bvh.nodes), 'channels': det.num_channels(),
                       'parallelism': 'photon-sharded x%d, geometry replicated' % world},
            'detail': {'kernel_ms_per_step': live['kernel_ms'] / args.steps,
                       'trace_ms_per_step': live['trace_ms'] / args.steps,
                       'launches_per_step': live['launches'] / args.steps,
                       'host_steps_per_propagate': live['host_steps'] / args.steps,
                       'detected_fraction': detected / args.photons,
                       'channel_hits_all_ranks': channel_hits},
            'roofline': None, 'cpu_baseline': None,
        }
        n = float(args.photons)
        ostats = None
        if not args.no_cpu_baseline and world == 1:
            threads = min(16, len(os.sched_getaffinity(0)))
            cpu, b_ref, ostats, nsample = cpu_baseline(PackedGeometry(det), photons, nslots, args.nthreads_per_block,
                                                   args.max_blocks, args.max_steps, args.seed, args.cpu_budget,
                                                   threads)
            result['cpu_baseline'] = cpu
            result['detail']['reference_bvh_nodes_per_photon'] = ostats['nodes_visited'] / nsample
            result['detail']['reference_bvh_triangles_per_photon'] = ostats['tris_tested'] / nsample
            result['detail']['bytes_per_photon_alg_8d'] = b_ref
        if live['trace_launches']:
            result['roofline'] = roofline(args, live, cst, ostats, n)
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
