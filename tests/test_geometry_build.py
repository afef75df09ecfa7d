"""The host geometry layer reproduces the reference's meshes bit for bit
(fixtures exported by tests/golden/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _names(objs):
    return np.array([('' if o is None else o.name) for o in objs])


def test_pmt_solid_matches_reference():
    from chroma.demo.pmt import build_8inch_pmt_with_lc
    p = build_8inch_pmt_with_lc()
    g = np.load(os.path.join(GOLDEN, 'pmt_lc_solid.npz'))
    assert np.array_equal(p.mesh.vertices, g['vertices'])
    assert np.array_equal(p.mesh.triangles, g['triangles'])
    for k in ('material1', 'material2', 'surface'):
        assert np.array_equal(_names(getattr(p, k)), g[k])
    assert np.array_equal(p.color, g['color'])


def test_cube_matches_reference():
    from chroma import make
    c = make.cube(1000.0)
    g = np.load(os.path.join(GOLDEN, 'cube_1000.npz'))
    assert np.array_equal(c.vertices, g['vertices']) and np.array_equal(c.triangles, g['triangles'])


def test_small_detector_flatten_matches_reference(small_detector):
    d = small_detector
    g = np.load(os.path.join(GOLDEN, 'detector_small.npz'))
    assert np.array_equal(d.mesh.vertices, g['vertices'])
    assert np.array_equal(d.mesh.triangles, g['triangles'])
    assert np.array_equal(d.solid_id, g['solid_id'])
    assert np.array_equal(d.colors, g['colors'])
    mn = _names(d.unique_materials)
    sn = _names(d.unique_surfaces)
    # index order may differ (the reference orders by set() hash), names must not
    assert np.array_equal(mn[d.material1_index], g['material_names'][g['material1_index']])
    assert np.array_equal(mn[d.material2_index], g['material_names'][g['material2_index']])
    s, gs = d.surface_index, g['surface_index']
    assert np.array_equal(s < 0, gs < 0)
    assert np.array_equal(sn[s[s >= 0]], g['surface_names'][gs[gs >= 0]])
    assert np.array_equal(d.solid_id_to_channel_index, g['solid_id_to_channel_index'])
    assert np.array_equal(d.time_cdf[1], g['time_cdf_y']) and np.array_equal(d.charge_cdf[0], g['charge_cdf_x'])


def test_tiny_detector_hashes():
    from chroma import demo
    h = json.load(open(os.path.join(GOLDEN, 'reference_hashes.json')))['tiny']
    t = demo.tiny()
    t.flatten()
    md5 = lambda a: hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()   # noqa: E731
    assert len(t.mesh.triangles) == h['triangles'] and len(t.mesh.vertices) == h['vertices']
    assert t.num_channels() == h['channels']
    assert md5(t.mesh.triangles.astype(np.int64)) == h['md5_triangles']
    assert md5(t.solid_id.astype(np.int64)) == h['md5_solid_id']
    assert float(t.mesh.vertices.astype(np.float64).sum()) == h['vertex_sum']


def test_from_film_matches_reference():
    from chroma import tools
    h = json.load(open(os.path.join(GOLDEN, 'reference_hashes.json')))
    pos, d = tools.from_film()
    m = hashlib.md5(np.asarray(pos, np.float64).tobytes())
    m.update(np.asarray(d, np.float64).tobytes())
    assert m.hexdigest() == h['from_film_md5']


def test_packing_tables(small_detector, small_packed):
    """Tables are np.interp onto 60..995 nm, float32, padded by one element."""
    from chroma.geometry import standard_wavelengths
    pk = small_packed
    assert len(pk.wavelengths) == 188 and pk.wavelength_step == 5.0
    for m, mp in zip(small_detector.unique_materials, pk.materials):
        ri = np.interp(standard_wavelengths, m.refractive_index[:, 0], m.refractive_index[:, 1]).astype(np.float32)
        assert np.array_equal(mp['refractive_index'][:-1], ri) and mp['refractive_index'][-1] == ri[-1]
    codes = pk.material_codes
    assert np.array_equal((codes >> 24) & 0xFF, small_detector.material1_index & 0xFF)
    assert np.array_equal((codes >> 8) & 0xFF, small_detector.surface_index & 0xFF)


def test_scintillator_detector_build():
    """chroma.demo.scint (BASELINE config 5): same PMT layout and mesh size as
    demo.tiny(), three light-cone surface models, a 2-component scintillator
    whose re-emission CDFs are proper CDFs."""
    from chroma.demo import scint
    det = scint.tiny()
    det.flatten()
    assert len(det.mesh.triangles) == 389568 and det.num_channels() == 53
    models = sorted({s.model for s in det.unique_surfaces if s is not None})
    assert models == [0, 2, 3]
    ls = det.detector_material
    assert len(ls.comp_reemission_prob) == 2
    for cdf in ls.comp_reemission_wvl_cdf + ls.comp_reemission_time_cdf:
        assert cdf[0, 1] == 0.0 and cdf[-1, 1] == 1.0 and (np.diff(cdf[:, 1]) >= 0).all()
    dp = [s for s in det.unique_surfaces if s is not None and s.model == 3][0].dichroic_props
    assert len(dp.angles) == len(dp.dichroic_reflect) == len(dp.dichroic_transmit)
    for r, t in zip(dp.dichroic_reflect, dp.dichroic_transmit):
        assert (r[:, 1] + t[:, 1] <= 1.0 + 1e-6).all()


def test_native_vertex_unique_equals_numpy():
    """Mesh.remove_duplicate_vertices through chr_unique_vertices (the flatten
    of large meshes) == numpy's np.unique over the rows: same sorted unique
    rows and inverse, with duplicates, negative values and -0.0 coordinates;
    a set of equal rows mixing +0.0 and -0.0 (numpy's kept row then depends on
    its sort) and NaN rows are refused and left to numpy."""
    import numpy as np
    from chroma import geometry
    rng = np.random.default_rng(7)
    v = (rng.integers(-40, 40, size=(200_000, 3)) * 0.25).astype(np.float32)
    v[v == 0] = np.float32(-0.0)                      # every zero negative: no mixed run
    t = rng.integers(0, len(v), size=(70_000, 3))
    rows = v.view([('', np.float32)] * 3)
    u, inv = np.unique(rows, return_inverse=True)
    got = geometry._native_unique(v)
    assert got is not None
    assert np.array_equal(got[0].view(np.uint32), u.view(np.float32).reshape(-1, 3).view(np.uint32))
    assert np.array_equal(got[1], inv.reshape(-1))
    m = geometry.Mesh(v, t, remove_duplicate_vertices=True)
    assert np.array_equal(m.triangles, inv.reshape(-1)[t])
    mixed = v.copy()
    mixed[:2] = [[0.0, 1.0, 2.0], [-0.0, 1.0, 2.0]]
    assert geometry._native_unique(mixed) is None
    nan = v.copy()
    nan[5, 1] = np.nan
    assert geometry._native_unique(nan) is None


@pytest.mark.parametrize('key,kw', [('demo_detector', {}),
                                    ('detector_29k', dict(pmt_radius=23780.0, sphere_radius=24280.0))])
def test_benchmark_geometry_matches_reference_generator(key, kw):
    """The bench geometries (C3 demo.detector() and the 29k-PMT headline
    detector) are the reference generator's bit for bit: MD5 of vertices,
    triangles, solid_id and solid_id_to_channel_index against the record
    tests/golden/make_golden_geometry.py wrote by building them with the
    reference's own chroma.demo / Geometry.flatten."""
    from chroma import demo
    want = json.load(open(os.path.join(GOLDEN, 'reference_hashes.json')))[key]
    assert want['params'] == kw
    got = demo.geometry_hashes(demo.detector(**kw))
    assert {k: got[k] for k in got} == {k: want[k] for k in got}
