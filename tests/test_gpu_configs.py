"""HIP vs oracle at the BASELINE configs' own scale, and the walks the bench
takes there.

* C2: 1,048,576 isotropic photons on demo.tiny() with Simulation's launch
  shape (512 x 1024): the first host step is split into trace + shade with
  the direction-binned trace order (n >= 2^20, propagate.hip kBinFirstMin).
* C3: 1,100,000 photons of the bench's own source on demo.detector()
  (58.96M triangles, 10,055 PMTs), same launch shape, max_steps 1000.
* Flat walks (a direction component of non-finite reciprocal: the reference
  slab test then skips that axis, intersect.h:121-144): decomposed into
  sub-walks by trace_kernel, walked whole by the tail kernel; both == oracle.
* The default walk vs the reference BVH walked in the reference's DFS order
  (CHR_PROPAGATE_VARIANT=1, tools/ab_variants.py) on the C3 workload.

Bit-exact on history flags, last-hit triangles and channels; floats within
1e-5 relative (they are bit-identical in practice).
"""
import importlib.util
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLOAT_RTOL = 1e-5


def _bench():
    spec = importlib.util.spec_from_file_location('bench_module', os.path.join(ROOT, 'bench.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    torch.cuda.set_device(0)


def _channels(flags, last_hit, solid_id, s2c):
    ch = np.full(len(flags), -1, np.int64)
    det = ((flags & 4) != 0) & (last_hit > -1)
    ch[det] = np.asarray(s2c, np.int64)[np.asarray(solid_id, np.int64)[last_hit[det]]]
    return ch


def _check(got, host, geo, label):
    assert np.array_equal(got.flags, host.flags), '%s: flags differ at %s' % (
        label, np.flatnonzero(got.flags != host.flags)[:8])
    assert np.array_equal(got.last_hit_triangles, host.last_hit_triangles), label + ': last hits differ'
    assert np.array_equal(_channels(got.flags, got.last_hit_triangles, geo.solid_id, geo.solid_id_to_channel_index),
                          _channels(host.flags, host.last_hit_triangles, geo.solid_id,
                                    geo.solid_id_to_channel_index)), label + ': channels differ'
    for f in ('pos', 'dir', 'pol', 't', 'wavelengths', 'weights'):
        a = getattr(got, f).astype(np.float64)
        b = getattr(host, f).astype(np.float64)
        scale = np.maximum(np.abs(b), 1.0 if f in ('pos', 'dir', 'pol') else 1e-30)
        assert np.all(np.abs(a - b) <= FLOAT_RTOL * scale), '%s: %s beyond %g' % (label, f, FLOAT_RTOL)


def _gpu_vs_oracle(geo, det_gpu, photons, ntpb, max_blocks, max_steps, seed=1, label=''):
    from chroma import gpu
    from chroma.gpu.packing import PackedGeometry
    nslots = ntpb * max_blocks
    gp = gpu.GPUPhotons(photons, copy_flags=True, copy_triangles=False, copy_weights=False)
    gp.propagate(det_gpu, gpu.get_rng_states(nslots, seed=seed), nthreads_per_block=ntpb, max_blocks=max_blocks,
                 max_steps=max_steps)
    stats = gp.last_stats
    got = gp.get()
    host = oracle.HostPhotons(photons)
    host.last_hit_triangles[:] = -1
    host.weights[:] = 1.0
    oracle.propagate(PackedGeometry(geo), host, oracle.rng_init(nslots, seed=seed), nslots, ntpb, max_blocks,
                     max_steps)
    _check(got, host, geo, label)
    return got, host, stats


def _flatten_some(photons, seed, nplane, naxis):
    """Give nplane photons a direction in a coordinate plane (one exactly-zero
    component), naxis photons one along an axis (two zeros) and one photon a
    denormal component."""
    rng = np.random.default_rng(seed)
    d = photons.dir.astype(np.float64).copy()
    n = len(d)
    idx = rng.permutation(n)
    plane, axis = idx[:nplane], idx[nplane: nplane + naxis]
    d[plane, rng.integers(0, 3, len(plane))] = 0.0
    ax = rng.integers(0, 3, len(axis))
    d[axis] = 0.0
    d[axis, ax] = rng.choice([-1.0, 1.0], len(axis))
    d /= np.linalg.norm(d, axis=1)[:, None]
    d = d.astype(np.float32)
    d[idx[-1]] = np.array([0.6, 0.8, 1e-40], np.float32)     # 1/1e-40 overflows: flat too
    r = rng.normal(size=(n, 3))
    p = np.cross(d.astype(np.float64), r)
    p /= np.linalg.norm(p, axis=1)[:, None]
    photons.dir[:] = d
    photons.pol[:] = p.astype(np.float32)
    return photons


@pytest.mark.parametrize('ntpb,max_blocks,max_steps', [(64, 64, 1000), (256, 1024, 1000)])
def test_flat_walks_small_detector(cuda, small_detector, ntpb, max_blocks, max_steps):
    """(64, 64): many one-step host steps -> flat walks in the trace pass;
    (256, 1024): one multi-step launch -> flat walks in the tail (both with the
    flat-axis slab test, propagate.hip make_slab)."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    photons = _flatten_some(isotropic(30000, seed=41), 41, 3750, 470)
    det = gpu.GPUDetector(small_detector)
    got, host, st = _gpu_vs_oracle(small_detector, det, photons, ntpb, max_blocks, max_steps,
                                   label='flat %dx%d' % (ntpb, max_blocks))
    if ntpb * max_blocks < 30000:
        assert st.flat_walks > 1000, st.flat_walks
    else:
        assert st.flat_walks_whole > 1000, st.flat_walks_whole


@pytest.fixture(scope='module')
def tiny_geo():
    from chroma import demo, loader
    return loader.create_geometry_from_obj(demo.tiny())


def test_c2_tiny_1m_binned_first_step(cuda, tiny_geo):
    """BASELINE config 2: 2^20 isotropic photons on demo.tiny(), launch shape
    512 x 1024 -> the binned split first step runs; HIP == oracle."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    n = 1 << 20
    photons = isotropic(n, seed=20260102)
    det = gpu.GPUDetector(tiny_geo)
    got, host, st = _gpu_vs_oracle(tiny_geo, det, photons, 512, 1024, 1000, label='C2 tiny 1M')
    assert st.trace_launches >= 1 and st.trace_rays >= n      # the split path (first step binned) ran
    assert st.stack_overflows == 0
    assert ((host.flags & 4) != 0).sum() > 1000


def test_c2_tiny_flat_walks(cuda, tiny_geo):
    """Flat walks at 1M photons on demo.tiny() (trace pass, flat-axis slab test)."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    photons = _flatten_some(isotropic(1 << 20, seed=5), 5, 2000, 200)
    det = gpu.GPUDetector(tiny_geo)
    got, host, st = _gpu_vs_oracle(tiny_geo, det, photons, 512, 1024, 1000, label='C2 tiny flat')
    assert st.flat_walks > 1500, st.flat_walks


@pytest.fixture(scope='module')
def demo_det():
    """demo.detector() through the bench's own builder (node-local cache
    shared with bench.py on the same box)."""
    b = _bench()
    return b.build_geometry('demo', os.environ.get('CHROMA_BENCH_CACHE', '/tmp/chroma_bench_cache'))


@pytest.mark.timeout(900)
def test_c3_demo_detector_parity(cuda, demo_det):
    """BASELINE config 3 (primary geometry): 1.1M photons of the bench source on
    demo.detector() (58.96M triangles), launch shape 512 x 1024, max_steps
    1000: HIP == oracle (split steps, binned first step, group-walk tail)."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    photons = isotropic(1_100_000, seed=20260102)
    det = gpu.GPUDetector(demo_det)
    got, host, st = _gpu_vs_oracle(demo_det, det, photons, 512, 1024, 1000, label='C3 demo 1.1M')
    assert st.trace_launches >= 2
    assert ((host.flags & 4) != 0).sum() > 10000


@pytest.mark.timeout(900)
def test_exact_order_walk_equals_default(cuda, demo_det, monkeypatch):
    """The reference BVH walked in the reference's DFS order (variant 1: the
    reference's node array, stack order and strict-'<' tie rule) gives the
    same photons as the default wide walk on the C3 workload."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    photons = isotropic(1_100_000, seed=20260102)
    det = gpu.GPUDetector(demo_det)
    out = {}
    for v in ('0', '1'):
        monkeypatch.setenv('CHR_PROPAGATE_VARIANT', v)
        gp = gpu.GPUPhotons(photons, copy_flags=True, copy_triangles=False, copy_weights=False)
        gp.propagate(det, gpu.get_rng_states(512 * 1024, seed=1), nthreads_per_block=512, max_blocks=1024,
                     max_steps=1000)
        out[v] = gp.get()
    a, b = out['0'], out['1']
    for f in ('flags', 'last_hit_triangles', 'pos', 'dir', 'pol', 't', 'wavelengths'):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
