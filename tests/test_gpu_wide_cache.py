"""The traversal-BVH cache on the device: a geometry
uploaded from the cached compact form propagates exactly the photons of one
whose traversal BVH was just built (and of the oracle), and occupies the same
HBM.  Reference: chroma/cache.py:209-236, chroma/loader.py:131-160 (the
reference caches the BVH its kernel walks)."""
import copy

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from chroma.gpu import create_cuda_context
    return create_cuda_context()


def _fields(gp):
    got = gp.get()
    return {f: getattr(got, f) for f in ('pos', 'dir', 'pol', 'wavelengths', 't', 'flags', 'last_hit_triangles',
                                         'weights')}


def test_cached_traversal_bvh_same_photons(cuda, tmp_path, small_detector, small_packed, monkeypatch):
    from chroma import gpu
    from chroma.cache import Cache
    from chroma.photon_source import isotropic
    cache = Cache(str(tmp_path))
    md5 = small_detector.mesh.md5()
    geos = []
    for i in range(2):
        g = copy.copy(small_detector)
        if i == 0:
            g.bvh = copy.copy(small_detector.bvh)
            g.bvh.wide = None
            cache.save_bvh(g.bvh, md5)           # a fresh cache: this one builds and saves
        else:
            g.bvh = cache.load_bvh(md5)          # a new BVH object from the cache: loads
        geos.append(g)
    gg = [gpu.GPUGeometry(g) for g in geos]
    assert gg[0].setup_times['wide_bvh_source'] == 'built'
    assert gg[1].setup_times['wide_bvh_source'] == 'cache'
    assert gg[0].device_bytes() == gg[1].device_bytes()
    photons = isotropic(200000, seed=77)
    out = []
    for g in gg:
        rng = gpu.get_rng_states(256 * 1024, seed=3)
        gp = gpu.GPUPhotons(photons, copy_flags=True, copy_triangles=False, copy_weights=False)
        gp.propagate(g, rng, nthreads_per_block=256, max_blocks=1024, max_steps=1000)
        out.append((_fields(gp), rng.get().reshape(-1)))
    for f in out[0][0]:
        assert np.array_equal(out[0][0][f].view(np.uint32), out[1][0][f].view(np.uint32)), f
    assert np.array_equal(out[0][1], out[1][1])
    # and the oracle's photons (the cache path is the product path of every later run)
    host = oracle.HostPhotons(photons)
    host.flags[:] = 0
    host.last_hit_triangles[:] = -1
    host.weights[:] = 1
    st = oracle.rng_init(256 * 1024, seed=3)
    oracle.propagate(small_packed, host, st, 256 * 1024, 256, 1024, 1000)
    assert np.array_equal(out[1][0]['flags'], host.flags)
    assert np.array_equal(out[1][0]['last_hit_triangles'], host.last_hit_triangles)
    assert np.array_equal(out[1][0]['pos'].view(np.uint32), host.pos.view(np.uint32))
    assert np.array_equal(out[1][1], st)


def test_corrupt_cache_refused_before_upload(cuda, tmp_path, small_detector):
    """A cached form that does not fit the geometry is refused by the library
    (CHR_ERR_INVALID) before any kernel could read out of bounds."""
    from chroma import gpu
    from chroma.gpu import _native, wide_bvh
    from chroma.gpu.packing import PackedGeometry
    packed = PackedGeometry(small_detector)
    w = wide_bvh.build(packed)
    bad = wide_bvh.WideBVH(w.nodes, np.array(w.rec_id), np.array(w.rec_rank), w.max_depth, w.usable,
                           w.leaf_max, w.key)
    bad.rec_id[3] = len(packed.triangles) + 5
    g = copy.copy(small_detector)
    g.bvh = copy.copy(small_detector.bvh)
    g.bvh.wide = bad
    with pytest.raises(_native.NativeError, match='wide BVH'):
        gpu.GPUGeometry(g)


def test_refused_cache_entry_rebuilt(cuda, tmp_path, small_detector):
    """a cache entry of the right shape whose contents the upload's
    validation refuses (a record id out of range) is dropped and the traversal
    BVH rebuilt once (setup source 'rebuilt'); the next geometry loads the
    rewritten entry from the cache."""
    from chroma import gpu
    from chroma.cache import Cache
    from chroma.gpu import wide_bvh
    cache = Cache(str(tmp_path))
    md5 = small_detector.mesh.md5()
    g0 = copy.copy(small_detector)
    g0.bvh = copy.copy(small_detector.bvh)
    g0.bvh.wide = None
    cache.save_bvh(g0.bvh, md5)
    assert gpu.GPUGeometry(g0).setup_times['wide_bvh_source'] == 'built'
    d = wide_bvh.directory(str(tmp_path), md5, 'default', wide_bvh.builder_key())
    rid = np.load(d + '/rec_id.npy')
    rid[3] = len(small_detector.mesh.triangles) + 5
    np.save(d + '/rec_id.npy', rid, allow_pickle=False)
    g1 = copy.copy(small_detector)
    g1.bvh = cache.load_bvh(md5)
    assert gpu.GPUGeometry(g1).setup_times['wide_bvh_source'] == 'rebuilt'
    g2 = copy.copy(small_detector)
    g2.bvh = cache.load_bvh(md5)
    assert gpu.GPUGeometry(g2).setup_times['wide_bvh_source'] == 'cache'
