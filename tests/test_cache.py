"""On-disk geometry/BVH cache (chroma.cache, reference chroma/cache.py:1-246)
and the loader paths that use it (reference chroma/loader.py:13-191)."""
import os

import numpy as np
import pytest

import scenes


def _packed_arrays(geo):
    """Everything the propagator consumes, as flat arrays (PackedGeometry)."""
    from chroma.gpu.packing import PackedGeometry
    pk = PackedGeometry(geo)
    out = {'vertices': pk.vertices, 'triangles': pk.triangles, 'nodes': pk.nodes,
           'world_origin': pk.world_origin, 'world_scale': np.asarray(pk.world_scale),
           'material_codes': pk.material_codes}
    for i, m in enumerate(pk.materials):
        for k, v in m.items():
            out['m%d.%s' % (i, k)] = np.asarray(v)
    for i, s in enumerate(pk.surfaces):
        for k, v in (s or {'none': 0}).items():
            out['s%d.%s' % (i, k)] = np.asarray(v)
    for i, p in enumerate(pk.wireplanes):
        for k, v in p.items():
            out['w%d.%s' % (i, k)] = np.asarray(v)
    return out


def test_geometry_and_bvh_round_trip(tmp_path):
    """Every surface model, multi-component bulk re-emission, wire planes and
    the detector channel maps survive save/load; the packed device arrays are
    identical."""
    from chroma.cache import Cache
    from chroma import loader
    det = loader.create_geometry_from_obj(scenes.physics_scene(), cache_dir=str(tmp_path))
    cache = Cache(str(tmp_path))
    md5 = det.mesh.md5()
    assert cache.exist_bvh(md5)                      # load_bvh saved it (update_bvh_cache)
    cache.save_geometry('scene', det)
    assert cache.list_geometry() == ['scene']
    assert cache.get_geometry_hash('scene') == md5

    got = cache.load_geometry('scene')
    got.bvh = cache.load_bvh(md5)
    assert type(got) is type(det)
    for k in ('solid_id_to_channel_index', 'channel_index_to_solid_id'):
        np.testing.assert_array_equal(getattr(got, k), getattr(det, k))
    for a, b in zip(got.time_cdf + got.charge_cdf, det.time_cdf + det.charge_cdf):
        np.testing.assert_array_equal(a, b)
    assert [s.model if s else None for s in got.unique_surfaces] == \
        [s.model if s else None for s in det.unique_surfaces]
    want, have = _packed_arrays(det), _packed_arrays(got)
    assert sorted(want) == sorted(have)
    for k in want:
        np.testing.assert_array_equal(have[k], want[k], err_msg=k)


def test_default_geometry_and_loader_string(tmp_path, small_detector):
    from chroma.cache import Cache, GeometryNotFoundError
    from chroma import loader
    cache = Cache(str(tmp_path))
    with pytest.raises(GeometryNotFoundError):
        cache.load_geometry('nope')
    with pytest.raises(GeometryNotFoundError):
        cache.set_default_geometry('nope')
    cache.save_geometry('small', small_detector)
    cache.set_default_geometry('small')
    assert os.path.islink(cache.get_geometry_filename('.default'))
    cache.set_default_geometry('small')              # replacing the symlink is fine
    # '' -> default geometry; BVH built and cached on the first load, read on the second
    g1 = loader.load_geometry_from_string('', cache_dir=str(tmp_path))
    assert cache.exist_bvh(g1.mesh.md5())
    g2 = loader.load_geometry_from_string('small', cache_dir=str(tmp_path))
    np.testing.assert_array_equal(g2.bvh.nodes, small_detector.bvh.nodes)
    np.testing.assert_array_equal(g1.mesh.triangles, small_detector.mesh.triangles)
    # named BVH missing and auto_build disabled -> None (reference loader.py:153-158)
    g3 = loader.load_geometry_from_string('small:other', auto_build_bvh=False, cache_dir=str(tmp_path))
    assert g3.bvh is None
    cache.remove_geometry('small')
    assert 'small' not in cache.list_geometry()
    cache.remove_bvh(g1.mesh.md5())
    assert not cache.exist_bvh(g1.mesh.md5())


def test_cache_files_load_without_pickle(tmp_path, small_detector):
    """Cache files are plain npz: np.load(allow_pickle=False) reads every entry."""
    from chroma.cache import Cache
    cache = Cache(str(tmp_path))
    cache.save_geometry('g', small_detector)
    cache.save_bvh(small_detector.bvh, small_detector.mesh.md5())
    for path in (cache.get_geometry_filename('g'), cache.get_bvh_filename(small_detector.mesh.md5())):
        with np.load(path, allow_pickle=False) as z:
            for k in z.files:
                assert z[k].dtype != object


def test_cache_dir_must_be_directory(tmp_path):
    from chroma.cache import Cache
    p = tmp_path / 'file'
    p.write_text('x')
    with pytest.raises(IOError):
        Cache(str(p))
