"""HIP vs oracle on the BASELINE configs that had no -m gpu parity test before
round 3, at their own sizes and launch shape (512 x 1024
= Simulation's, max_steps 1000), through the bench's geometry builder:

* C5: chroma.demo.scint.detector() at full size (58.96M triangles: liquid
  scintillator with 2-component bulk re-emission, light cones cycling shiny /
  dichroic / WLS), >= 2^20 photons so the binned first step runs -- the
  surfaces of reference photon.h:518-532 (bulk re-emission) and 829-907 (WLS,
  dichroic) on the geometry the C5 bench line measures;
* C4: the shard rank 7 of an 8-GPU run propagates (photon seed 20260102+7,
  RNG subsequences 7*524288 + slot, bench.py rng_first_subsequence) on
  demo.detector(), 1.1M photons, sequential and pipelined (two batches);
* C4's rank 7 on the 29k-PMT geometry with a first batch of 2^20 + 50,000
  photons: the binned first step under first_subsequence = 7*524288;
* C3 29k-PMT variant (the headline geometry, 169.9M triangles) at 1.1M photons.

Bit-exact on history flags, last-hit triangles and channels; floats within
1e-5 relative (bit-identical in practice).
"""
import importlib.util
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NTPB, MAXB, STEPS = 512, 1024, 1000
NSLOTS = NTPB * MAXB
PHOTON_SEED = 20260102
FLOAT_RTOL = 1e-5


def _bench():
    spec = importlib.util.spec_from_file_location('bench_module', os.path.join(ROOT, 'bench.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _geometry(name):
    return _bench().build_geometry(name, os.environ.get('CHROMA_BENCH_CACHE', '/tmp/chroma_bench_cache'))


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    torch.cuda.set_device(0)


def _channels(flags, last_hit, geo):
    ch = np.full(len(flags), -1, np.int64)
    det = ((flags & 4) != 0) & (last_hit > -1)
    ch[det] = np.asarray(geo.solid_id_to_channel_index, np.int64)[np.asarray(geo.solid_id, np.int64)[last_hit[det]]]
    return ch


def _check(got, host, geo, label):
    bad = np.flatnonzero(got.flags != host.flags)
    assert bad.size == 0, '%s: %d flags differ, first at %s' % (label, bad.size, bad[:8])
    assert np.array_equal(got.last_hit_triangles, host.last_hit_triangles), label + ': last hits differ'
    assert np.array_equal(_channels(got.flags, got.last_hit_triangles, geo),
                          _channels(host.flags, host.last_hit_triangles, geo)), label + ': channels differ'
    for f in ('pos', 'dir', 'pol', 't', 'wavelengths', 'weights'):
        a = getattr(got, f).astype(np.float64)
        b = getattr(host, f).astype(np.float64)
        scale = np.maximum(np.abs(b), 1.0 if f in ('pos', 'dir', 'pol') else 1e-30)
        assert np.all(np.abs(a - b) <= FLOAT_RTOL * scale), '%s: %s beyond %g' % (label, f, FLOAT_RTOL)


def _oracle(geo, batches, first_subsequence):
    """The oracle on the batches in order, one RNG state set (as propagate
    calls in sequence)."""
    from chroma.gpu.packing import PackedGeometry
    packed = PackedGeometry(geo)
    st = oracle.rng_init(NSLOTS, seed=1, first_subsequence=first_subsequence)
    hosts = []
    for photons in batches:
        host = oracle.HostPhotons(photons)
        host.last_hit_triangles[:] = -1
        host.weights[:] = 1.0
        oracle.propagate(packed, host, st, NSLOTS, NTPB, MAXB, STEPS)
        hosts.append(host)
    return hosts, st


def _gpu(det_gpu, batches, first_subsequence, pipelined):
    from chroma import gpu
    gps = [gpu.GPUPhotons(p, copy_flags=True, copy_triangles=False, copy_weights=False) for p in batches]
    rng = gpu.get_rng_states(NSLOTS, seed=1, first_subsequence=first_subsequence)
    kw = dict(nthreads_per_block=NTPB, max_blocks=MAXB, max_steps=STEPS)
    if pipelined:
        stats = gpu.propagate_batches(gps, det_gpu, rng, **kw)
    else:
        stats = []
        for gp in gps:
            gp.propagate(det_gpu, rng, **kw)
            stats.append(gp.last_stats)
    return [gp.get() for gp in gps], rng.get(), stats


@pytest.mark.timeout(1200)
def test_c5_scint_detector_full_size(cuda):
    """C5 at full size, 2^20 + 50,000 photons: HIP == oracle, with the bulk
    re-emission (BULK_REEMIT), WLS re-emission (SURFACE_REEMIT), dichroic /
    WLS transmission and detection branches all taken."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    geo = _geometry('scint')
    assert len(geo.mesh.triangles) > 50_000_000
    photons = isotropic((1 << 20) + 50_000, seed=PHOTON_SEED)
    got, rng, stats = _gpu(gpu.GPUDetector(geo), [photons], 0, pipelined=False)
    hosts, st = _oracle(geo, [photons], 0)
    _check(got[0], hosts[0], geo, 'C5 scint full')
    assert np.array_equal(rng.reshape(-1), st.reshape(-1))
    assert stats[0].trace_launches >= 1 and stats[0].stack_overflows == 0
    fl = hosts[0].flags
    for bit, name in ((1 << 9, 'BULK_REEMIT'), (1 << 7, 'SURFACE_REEMIT'), (1 << 8, 'SURFACE_TRANSMIT'),
                      (1 << 2, 'SURFACE_DETECT'), (1 << 6, 'REFLECT_SPECULAR')):
        assert ((fl & bit) != 0).sum() > 100, '%s (bit %d) not exercised' % (name, bit)


@pytest.fixture(scope='module')
def demo_geo():
    return _geometry('demo')


@pytest.mark.timeout(900)
@pytest.mark.parametrize('pipelined', [False, True])
def test_c4_rank7_shard(cuda, demo_geo, pipelined):
    """C4's rank 7 on demo.detector(): its own photon seed and RNG
    subsequences [7*524288, 8*524288); 1.1M photons as two batches (the
    second batch continues the first's RNG states), propagated one call each
    or pipelined by propagate_batches; HIP == oracle."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    rank = 7
    first = _bench().rng_first_subsequence(rank, NSLOTS)
    assert first == 7 * 524288
    photons = isotropic(1_100_000, seed=PHOTON_SEED + rank)
    batches = [photons[:600_000], photons[600_000:]]
    got, rng, stats = _gpu(gpu.GPUDetector(demo_geo), batches, first, pipelined)
    hosts, st = _oracle(demo_geo, batches, first)
    for i in range(2):
        _check(got[i], hosts[i], demo_geo, 'C4 rank 7 batch %d (%s)' % (i, 'pipelined' if pipelined else 'sequential'))
    assert np.array_equal(rng.reshape(-1), st.reshape(-1))
    assert all(s.trace_launches >= 1 for s in stats)


@pytest.fixture(scope='module')
def geo29k():
    return _geometry('29k')


@pytest.mark.timeout(1200)
@pytest.mark.parametrize('pipelined', [False, True])
def test_c4_rank7_shard_29k(cuda, geo29k, pipelined):
    """C4's rank 7 on the headline geometry (29,007 PMTs): its own photon seed
    and RNG subsequences from 7*524288, a first batch of 2^20 + 50,000 photons
    -- so the direction-binned first step runs under the rank's non-zero
    first_subsequence -- then a second batch of 200,000 continuing its RNG
    states; one propagate call each or pipelined; HIP == oracle."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    rank = 7
    first = _bench().rng_first_subsequence(rank, NSLOTS)
    assert first == 7 * 524288
    n0 = (1 << 20) + 50_000
    photons = isotropic(n0 + 200_000, seed=PHOTON_SEED + rank)
    batches = [photons[:n0], photons[n0:]]
    got, rng, stats = _gpu(gpu.GPUDetector(geo29k), batches, first, pipelined)
    hosts, st = _oracle(geo29k, batches, first)
    for i in range(2):
        _check(got[i], hosts[i], geo29k, 'C4 29k rank 7 batch %d (%s)' % (i, 'pipelined' if pipelined else 'sequential'))
    assert np.array_equal(rng.reshape(-1), st.reshape(-1))
    assert stats[0].trace_launches >= 1 and all(s.stack_overflows == 0 for s in stats)
    assert ((hosts[0].flags & 4) != 0).sum() > 10000


@pytest.mark.timeout(1200)
def test_c3_29k_detector_parity(cuda, geo29k):
    """The headline geometry (29,007 PMTs, 169.9M triangles) at 1.1M photons
    of the bench source: HIP == oracle."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    geo = geo29k
    assert geo.num_channels() == 29007
    photons = isotropic(1_100_000, seed=PHOTON_SEED)
    got, rng, stats = _gpu(gpu.GPUDetector(geo), [photons], 0, pipelined=False)
    hosts, st = _oracle(geo, [photons], 0)
    _check(got[0], hosts[0], geo, 'C3 29k 1.1M')
    assert np.array_equal(rng.reshape(-1), st.reshape(-1))
    assert ((hosts[0].flags & 4) != 0).sum() > 10000


# BENCH_r05's parity failure: photon 9,043,377 of the bench's
# 9,897,030-photon parity sample, batch 1, second step (tools/parity_watch.py,
# profiles/r06/parity_watch).  Its ray meets triangle 30,327,113 only through a
# float32 Moller-Trumbore false positive: the hit is reported at 36,510.26 mm
# while the exact ray meets that triangle's plane 7% outside it and enters the
# triangle's reference leaf box only at 36,511.24 mm.  The reference DFS meets it
# first and keeps it (the neighbour at 36,510.91 mm does not replace it); round 5's
# walks culled its box against the neighbour and returned the neighbour.
FP_ORIGIN = (-1942.692138671875, 16390.626953125, -1976.0341796875)
FP_DIR = (-0.24864476919174194, -0.8455895781517029, 0.47239193320274353)
FP_TRIANGLE, FP_DISTANCE = 30327113, 36510.26171875


@pytest.mark.timeout(1200)
def test_false_positive_hit_29k(cuda, geo29k):
    """The false-positive ray on every GPU walker, against the oracle (the
    reference DFS): the one-step launch's trace_kernel (2^17 copies: binned
    first step), the tail kernel (4,000 copies: grouped walks, walk_lone and
    the pair walk), the fused walk of distance_to_mesh, and walk_lone / the
    pair walk / the pair walk with lost handshakes in isolation."""
    import ctypes
    import torch
    from chroma import gpu
    from chroma.event import Photons
    from chroma.gpu import _native, gpuarray as ga, wide_bvh
    from chroma.gpu.packing import PackedGeometry
    from chroma.gpu.tools import current_stream
    packed = PackedGeometry(geo29k)
    o = np.array([FP_ORIGIN], np.float32)
    d = np.array([FP_DIR], np.float32)
    dist, tri = oracle.intersect_rays(packed, o, d, np.array([-1], np.int32))
    assert (int(tri[0]), float(dist[0])) == (FP_TRIANGLE, FP_DISTANCE)   # the oracle pinned on this ray
    gdet = gpu.GPUDetector(geo29k)
    # whole steps: HIP == oracle on copies of the ray (one step, every copy its own RNG slot)
    for n in (1 << 17, 4000):
        ph = Photons(np.repeat(o, n, 0), np.repeat(d, n, 0), np.tile(np.float32([[1, 0, 0]]), (n, 1)),
                     np.full(n, 420.0, np.float32))
        gp = gpu.GPUPhotons(ph, copy_flags=True, copy_triangles=False, copy_weights=False)
        rng = gpu.get_rng_states(NSLOTS, seed=1)
        gp.propagate(gdet, rng, nthreads_per_block=NTPB, max_blocks=MAXB, max_steps=1)
        got = gp.get()
        host = oracle.HostPhotons(ph)
        host.last_hit_triangles[:] = -1
        host.weights[:] = 1.0
        oracle.propagate(packed, host, oracle.rng_init(NSLOTS, seed=1), NSLOTS, NTPB, MAXB, 1)
        _check(got, host, geo29k, 'false-positive ray x %d' % n)
        # the false-positive hit decides the photon's bulk material (material1 = 1 from that
        # triangle's side, 1.75 m absorption length): nearly every copy is absorbed on the
        # way, against ~30% with the neighbour's (water, 104 m)
        assert ((host.flags & 2) != 0).sum() > 0.9 * n
    # the fused walk (distance_to_mesh)
    dd = ga.to_gpu(np.full(1, -7.0, np.float32))
    go, gd = ga.to_gpu(o.reshape(-1)), ga.to_gpu(d.reshape(-1))   # held: the call reads them asynchronously
    _native.call('chr_distance_to_mesh', gdet._handle, 1, go.gpudata, gd.gpudata, dd.gpudata, current_stream())
    torch.cuda.synchronize()
    assert float(dd.get()[0]) == FP_DISTANCE
    # walk_lone, the pair walk, the pair walk losing its handshakes
    wide, _ = wide_bvh.obtain(geo29k.bvh, gdet.packed)
    rays = np.zeros((64, 7), np.float32)
    rays[:, 0:3] = o
    rays[:, 3:6] = d
    rays[:, 6] = np.int32(-1).view(np.float32)
    dr = ga.to_gpu(rays.reshape(-1))
    for walker in (0, 1, 2):
        res = ga.zeros(64 * 4 + 1, np.uint32)
        _native.call('chr_walk_lone_timing', gdet._handle, dr.gpudata, 64, 1, 8, walker, res.gpudata,
                     current_stream())
        torch.cuda.synchronize()
        recs = res.get()[:-1].reshape(64, 4)[:, 0].view(np.int32)
        assert np.all(np.asarray(wide.rec_id)[recs] == FP_TRIANGLE), 'walker %d' % walker
