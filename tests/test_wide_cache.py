"""The traversal-BVH cache (chroma.gpu.wide_bvh): the
compact form a cache stores rebuilds exactly the 64-byte triangle records of
the full host build, a corrupt compact form is refused before anything
reaches the device, and the cache next to the reference BVH is found by a
BVH loaded from the same cache (reference chroma/cache.py:209-236,
chroma/loader.py:131-160).  The device upload of a cached form is checked
against a built one on the GPU (tests/test_gpu_wide_cache.py)."""
import ctypes
import os

import numpy as np
import pytest


def _full_and_compact(packed):
    from chroma.bvh.wide import build_wide_bvh
    from chroma.gpu import wide_bvh
    return build_wide_bvh(packed), wide_bvh.build(packed)


def _check_records(w, full, packed):
    """The compact form's records (the upload's) against the full build's: every word
    but the last (pad) equal; the upload's pad word is the record's leaf node
    (walk_up's start, wide_bvh.h).  Returns the records."""
    rec = w.records(packed)
    words = rec.reshape(-1).view(np.uint32).reshape(-1, 16)
    assert np.array_equal(words[:, :15], full.tris.view(np.uint8).reshape(-1).view(np.uint32).reshape(-1, 16)[:, :15])
    nodes = w.nodes.view(np.uint8).reshape(-1, 96)
    kinds, offs = nodes[:, 72:80].astype(np.int64), nodes[:, 80:88].astype(np.int64)
    tri_base = nodes[:, 68:72].copy().view(np.uint32).reshape(-1).astype(np.int64)
    leaf_of = np.full(len(words), -1, np.int64)
    for k in range(8):
        for t in range(4):
            m = (kinds[:, k] >= 1) & (kinds[:, k] <= 4) & (t < kinds[:, k])
            leaf_of[tri_base[m] + offs[m, k] + t] = np.flatnonzero(m)
    assert np.all(leaf_of >= 0) and np.array_equal(words[:, 15], leaf_of)
    return rec


def test_compact_rebuilds_records(small_packed):
    full, w = _full_and_compact(small_packed)
    assert w.usable and len(w.nodes) == len(full.nodes) and len(w.rec_id) == len(full.tris)
    assert np.array_equal(w.nodes.view(np.uint8).reshape(-1), full.nodes.view(np.uint8).reshape(-1))
    assert np.array_equal(w.rec_id, full.tris['id']) and np.array_equal(w.rec_rank, full.tris['rank'])
    rec = _check_records(w, full, small_packed)
    # a sub-range, as the upload fills it chunk by chunk
    n = len(w.rec_id)
    part = w.records(small_packed, first=n // 3, n=n // 4)
    assert np.array_equal(part, rec[n // 3:n // 3 + n // 4])
    assert w.leaf_max == 3 and w.key == 'w2-l3'


def test_compact_physics_scene():
    import scenes
    from chroma import loader
    from chroma.gpu.packing import PackedGeometry
    packed = PackedGeometry(loader.create_geometry_from_obj(scenes.physics_scene()))
    full, w = _full_and_compact(packed)
    _check_records(w, full, packed)


def _corrupt(w, **changes):
    from chroma.gpu.wide_bvh import WideBVH
    arrs = {k: np.array(getattr(w, k), copy=True) for k in ('nodes', 'rec_id', 'rec_rank')}
    for k, f in changes.items():
        f(arrs[k])
    return WideBVH(arrs['nodes'], arrs['rec_id'], arrs['rec_rank'], w.max_depth, w.usable, w.leaf_max, w.key)


@pytest.mark.parametrize('what', ['rank_dup', 'rank_range', 'id_range', 'inner_child', 'leaf_range', 'kind',
                                  'backward_child'])
def test_corrupt_compact_form_refused(small_packed, what):
    from chroma.gpu import _native, wide_bvh
    w = wide_bvh.build(small_packed)
    ntri = len(small_packed.triangles)

    def node_field(a, off, val):       # first inner node's kind / off / child_base bytes
        nodes = a.view(np.uint8).reshape(-1, 96)
        nodes[0, off] = val

    def child_base(a, val):
        a.view(np.uint8).reshape(-1, 96)[0, 64:68] = np.frombuffer(np.uint32(val).tobytes(), np.uint8)

    bad = {
        'rank_dup': dict(rec_rank=lambda a: a.__setitem__(1, a[0])),
        'rank_range': dict(rec_rank=lambda a: a.__setitem__(0, len(a))),
        'id_range': dict(rec_id=lambda a: a.__setitem__(5, ntri)),
        'inner_child': dict(nodes=lambda a: child_base(a, len(w.nodes) + 3)),
        'leaf_range': dict(nodes=lambda a: a.view(np.uint8).reshape(-1, 96).__setitem__(
            (len(w.nodes) - 1, slice(68, 72)), np.frombuffer(np.uint32(len(w.rec_id)).tobytes(), np.uint8))),
        'kind': dict(nodes=lambda a: node_field(a, 72, 9)),
        'backward_child': dict(nodes=lambda a: child_base(a, 0)),
    }[what]
    c = _corrupt(w, **bad)
    with pytest.raises(_native.NativeError, match='wide BVH'):
        c.records(small_packed, 0, 1)


def test_cache_round_trip(tmp_path, small_detector):
    """obtain(): built and saved next to the reference BVH, then found by a BVH
    loaded from the same cache; a different reference BVH is not served."""
    from chroma.cache import Cache
    from chroma.gpu import wide_bvh
    from chroma.gpu.packing import PackedGeometry
    cache = Cache(str(tmp_path))
    md5 = small_detector.mesh.md5()
    import copy
    geo = copy.copy(small_detector)
    geo.bvh = copy.copy(small_detector.bvh)
    cache.save_bvh(geo.bvh, md5)
    assert geo.bvh.cache_ref == (str(tmp_path), md5, 'default')
    packed = PackedGeometry(geo)
    w1, src1 = wide_bvh.obtain(geo.bvh, packed)
    assert src1 == 'built'
    d = wide_bvh.directory(str(tmp_path), md5, 'default', wide_bvh.builder_key())
    assert sorted(os.listdir(d)) == ['meta.json', 'nodes.npy', 'rec_id.npy', 'rec_rank.npy']
    assert cache.list_bvh(md5) == ['default']          # the .wide directory is not a BVH
    assert wide_bvh.obtain(geo.bvh, packed)[1] == 'memory'
    bvh2 = cache.load_bvh(md5)
    w2, src2 = wide_bvh.obtain(bvh2, packed)
    assert src2 == 'cache'
    for k in ('nodes', 'rec_id', 'rec_rank'):
        assert np.array_equal(np.asarray(getattr(w1, k)), np.asarray(getattr(w2, k)))
    assert np.array_equal(w2.records(packed), wide_bvh.build(packed).records(packed))
    # another reference BVH under the same name: the fingerprint no longer matches
    bvh3 = cache.load_bvh(md5)
    bvh3.nodes = np.array(bvh3.nodes, copy=True)
    bvh3.nodes.view(np.uint32).reshape(-1, 4)[-1, 0] ^= 1
    assert wide_bvh.load(str(tmp_path), md5, 'default', wide_bvh.builder_key(), wide_bvh.fingerprint(bvh3)) is None
    cache.remove_bvh(md5)
    assert not os.path.exists(os.path.dirname(d))


def test_cache_disabled(tmp_path, small_detector, monkeypatch):
    from chroma.cache import Cache
    from chroma.gpu import wide_bvh
    from chroma.gpu.packing import PackedGeometry
    import copy
    monkeypatch.setenv('CHROMA_WIDE_CACHE', '0')
    bvh = copy.copy(small_detector.bvh)
    Cache(str(tmp_path)).save_bvh(bvh, 'x' * 32)
    geo = copy.copy(small_detector)
    geo.bvh = bvh
    assert wide_bvh.obtain(bvh, PackedGeometry(geo))[1] == 'built'
    assert not os.path.exists(os.path.join(str(tmp_path), 'bvh', 'x' * 32, 'default.wide'))


def test_host_threads():
    from chroma.gpu import _native
    default = _native.host_threads()
    assert default >= 1
    try:
        _native.set_host_threads(3)
        assert _native.host_threads() == 3
    finally:
        _native.set_host_threads(0)
    assert _native.host_threads() == default
    with pytest.raises(_native.NativeError):
        _native.set_host_threads(-1)


def _saved(tmp_path, small_detector):
    import copy
    from chroma.cache import Cache
    from chroma.gpu import wide_bvh
    from chroma.gpu.packing import PackedGeometry
    cache = Cache(str(tmp_path))
    md5 = small_detector.mesh.md5()
    geo = copy.copy(small_detector)
    geo.bvh = copy.copy(small_detector.bvh)
    cache.save_bvh(geo.bvh, md5)
    packed = PackedGeometry(geo)
    assert wide_bvh.obtain(geo.bvh, packed)[1] == 'built'
    return cache, md5, geo, packed, wide_bvh.directory(str(tmp_path), md5, 'default', wide_bvh.builder_key())


@pytest.mark.parametrize('what', ['node_width', 'node_dtype', 'rank_length', 'id_dtype'])
def test_cache_entry_of_wrong_shape_is_rebuilt(tmp_path, small_detector, what):
    """load() checks the cached arrays before the C side reads
    nnodes * 96 node bytes and nrec ids / ranks; an entry of the wrong type or
    shape is not served (obtain() builds instead)."""
    from chroma.gpu import wide_bvh
    cache, md5, geo, packed, d = _saved(tmp_path, small_detector)
    f = {'node_width': 'nodes', 'node_dtype': 'nodes', 'rank_length': 'rec_rank', 'id_dtype': 'rec_id'}[what]
    a = np.load(os.path.join(d, f + '.npy'))
    a = {'node_width': lambda: a[:, :95], 'node_dtype': lambda: a.astype(np.uint16),
         'rank_length': lambda: a[:-1], 'id_dtype': lambda: a.astype(np.int64)}[what]()
    np.save(os.path.join(d, f + '.npy'), np.ascontiguousarray(a), allow_pickle=False)
    key, fp = wide_bvh.builder_key(), wide_bvh.fingerprint(geo.bvh)
    assert wide_bvh.load(str(tmp_path), md5, 'default', key, fp) is None
    bvh2 = cache.load_bvh(md5)
    assert wide_bvh.obtain(bvh2, packed)[1] == 'built'
    assert wide_bvh.load(str(tmp_path), md5, 'default', key, fp) is not None   # rewritten whole


def test_fingerprint_covers_every_node(small_detector):
    """A reference BVH that differs from the cached one's in a single node
    (any node, not only a sampled one) has another fingerprint."""
    import copy
    from chroma.gpu import wide_bvh
    bvh = copy.copy(small_detector.bvh)
    fp = wide_bvh.fingerprint(bvh)
    n = len(bvh.nodes)
    for i in (1, n // 2 + 1, n - 2):
        b = copy.copy(bvh)
        b.nodes = np.array(bvh.nodes, copy=True)
        b.nodes.view(np.uint32).reshape(-1, 4)[i, 3] ^= 1
        assert wide_bvh.fingerprint(b) != fp


def test_save_bvh_drops_derived_traversal_bvh(tmp_path, small_detector):
    """Cache.save_bvh over an existing BVH removes the traversal BVHs derived
    from the old one (<name>.wide/), as remove_bvh does."""
    cache, md5, geo, packed, d = _saved(tmp_path, small_detector)
    assert os.path.isdir(d)
    cache.save_bvh(geo.bvh, md5)
    assert not os.path.exists(os.path.dirname(d))
