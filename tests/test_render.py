"""The renderer's CPU oracle (oracle/chroma_oracle.c orc_render: render.cu
restated with the reference BVH walked in the reference order and the
sorting.h searchsorted / insert list) checked against independent facts:
the nearest entry is the oracle's own nearest-hit walk (mesh.h, a separate
code path), lists are sorted and hold every hit up to alpha_depth, misses
take the background colour, and the ARGB compositing of render.cu:150-179
recomputed in numpy from the kept entries gives the same pixels."""
import numpy as np

import oracle
from scenes import camera_rays


def _scene(cube_geometry):
    from chroma.gpu.packing import PackedGeometry
    packed = PackedGeometry(cube_geometry)
    colors = np.asarray(cube_geometry.colors, np.uint32)
    return packed, colors


def test_render_nearest_entry_is_the_nearest_hit(cube_geometry):
    packed, colors = _scene(cube_geometry)
    pos, d = camera_rays(48, 32, (2500.0, -3000.0, 1200.0), (0.0, 0.0, 0.0))
    pix, dx, dxlen, _ = oracle.render(packed, pos, d, colors, alpha_depth=1, bg_color=0xFF102030)
    dist, tri, _ = oracle.distance_to_mesh(packed, pos, d)
    hit = tri >= 0
    assert hit.any() and (~hit).any()
    assert np.array_equal(dxlen > 0, hit)
    # distance_to_mesh renormalises the direction (mesh.h callers do), render does not
    assert np.allclose(dx[hit], dist[hit], rtol=1e-6, atol=0)
    assert np.all(pix[~hit] == 0xFF102030)


def test_render_lists_sorted_and_complete(cube_geometry):
    packed, colors = _scene(cube_geometry)
    pos, d = camera_rays(40, 40, (2500.0, -3000.0, 1200.0), (0.0, 0.0, 0.0))
    depth = 6
    _, dx, dxlen, _ = oracle.render(packed, pos, d, colors, alpha_depth=depth)
    dx = dx.reshape(-1, depth)
    _, dx1, _, _ = oracle.render(packed, pos, d, colors, alpha_depth=1)
    for i in np.flatnonzero(dxlen):
        row = dx[i, :dxlen[i]]
        assert np.all(np.diff(row) >= 0)
        assert row[0] == dx1[i]
    # a convex cube: a ray through it crosses two faces (an edge-on ray may list both
    # triangles of a face)
    assert set(np.unique(dxlen)) <= {0, 2, 3, 4}
    assert (dxlen == 2).sum() > 100


def test_render_compositing(cube_geometry):
    """render.cu:150-179 from the kept entries, in float64 (within one 8-bit step)."""
    packed, colors = _scene(cube_geometry)
    colors = (np.arange(len(colors), dtype=np.uint32) * 0x00113355 + 0x40000000) & 0xFFFFFFFF   # partly transparent
    pos, d = camera_rays(32, 32, (2500.0, -3000.0, 1200.0), (0.0, 0.0, 0.0))
    depth, bg = 4, 0x80FFFFFF
    pix, dx, dxlen, col = oracle.render(packed, pos, d, colors, alpha_depth=depth, bg_color=bg)
    col = col.reshape(-1, depth, 4).astype(np.float64)
    for i in np.flatnonzero(dxlen):
        n = dxlen[i]
        scale, f = 1.0, np.zeros(3)
        for k in range(n):
            f += scale * col[i, k, :3] * col[i, k, 3]
            scale *= 1 - col[i, k, 3]
        a = float(np.float32(0x80 / 255.0))
        f += scale * np.array([0xFF, 0xFF, 0xFF]) * a
        scale *= 1 - a
        want = [255 if n >= depth else int(np.floor(255 * (1 - scale)))] + [int(np.floor(x / (1 - scale))) for x in f]
        got = [(int(pix[i]) >> s) & 0xFF for s in (24, 16, 8, 0)]
        assert all(abs(g - w) <= 1 for g, w in zip(got, want)), (i, got, want)


def test_render_keep_last_render_merges(cube_geometry):
    """A second render with the list kept merges its hits into it: the same
    rays again give every distance twice (capped at alpha_depth)."""
    packed, colors = _scene(cube_geometry)
    pos, d = camera_rays(24, 24, (2500.0, -3000.0, 1200.0), (0.0, 0.0, 0.0))
    depth = 8
    _, dx, dxlen, col = oracle.render(packed, pos, d, colors, alpha_depth=depth)
    first = dx.reshape(-1, depth).copy(), dxlen.copy()
    _, dx, dxlen, col = oracle.render(packed, pos, d, colors, alpha_depth=depth, dx=dx, dxlen=dxlen, color=col)
    dx = dx.reshape(-1, depth)
    for i in np.flatnonzero(first[1]):
        n = first[1][i]
        assert dxlen[i] == min(depth, 2 * n)
        assert np.array_equal(dx[i, :dxlen[i]], np.repeat(first[0][i, :n], 2)[:dxlen[i]])


def test_transform_matches_numpy():
    from chroma.transform import rotate
    r = np.random.default_rng(3)
    a = r.normal(size=(1000, 3)).astype(np.float32) * 100
    axis = np.array([0.3, -0.5, 0.81], np.float32)
    axis /= np.linalg.norm(axis)
    got = oracle.transform(a, 1, phi=0.7, axis=axis)
    assert np.allclose(got, rotate(a.astype(np.float64), 0.7, axis.astype(np.float64)), atol=1e-3)
    pt = np.array([10.0, -20.0, 5.0], np.float32)
    got = oracle.transform(a, 2, phi=-1.1, axis=axis, v=pt)
    want = rotate((a - pt).astype(np.float64), -1.1, axis.astype(np.float64)) + pt
    assert np.allclose(got, want, atol=1e-3)
    assert np.array_equal(oracle.transform(a, 0, v=pt), a + pt)


def test_hybrid_process_image():
    img = np.array([0.5, 2.0, -1.0, 0.25, 0.25, 0.999], np.float32)
    pix = oracle.hybrid_process_image(img, 1)
    assert pix[0] == (0xFF << 24 | 127 << 16 | 255 << 8 | 0)
    assert pix[1] == (0xFF << 24 | 63 << 16 | 63 << 8 | 254)
