"""HIP renderer (csrc/render.hip through GPURays and the C ABI) against the
CPU oracle's restatement of render.cu / transform.cu / hybrid_render.cu.

Render: pixels, kept-entry counts, distances and colours bit-exact (the HIP
kernel walks the wide BVH and inserts under (distance, reference rank); the
oracle walks the reference BVH in reference order with searchsorted insertion
-- the two must agree entry for entry), including keep_last_render merges of
rotated rays.  Transforms bit-exact.  Hybrid: RNG states after the lookup
pass bit-exact; the lookup sums within 1e-5 relative (float atomic adds on the
device, id order in the oracle; the reference's atomicExch loop is unordered
too); the image pass and process_image bit-exact from the same lookups."""
import numpy as np
import pytest

import oracle
from scenes import camera_rays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from chroma.gpu import create_cuda_context
    return create_cuda_context()


def _colors(geometry, transparent):
    c = np.asarray(geometry.colors, np.uint32)
    if transparent:    # vary colour and alpha per triangle so the compositing matters
        c = ((np.arange(len(c), dtype=np.uint64) * 0x00173359 + 0x30000000) & 0xFFFFFFFF).astype(np.uint32)
    return c


def _compare(rays, pix, want, depth):
    wpix, wdx, wlen, wcol = want
    n = len(wpix)
    assert np.array_equal(pix.get(), wpix)
    ln = rays.dxlen.get()
    assert np.array_equal(ln, wlen)
    # entries of ray i at [i * alpha_depth, (i + 1) * alpha_depth) (render.cu:84-85)
    dx = rays.dx.get()[:n * depth].reshape(n, depth)
    col = rays.color.get().view(np.float32)[:4 * n * depth].reshape(n, depth, 4)
    wdx = wdx.reshape(n, depth)
    wcol = wcol.reshape(n, depth, 4)
    for i in np.flatnonzero(ln):
        assert np.array_equal(dx[i, :ln[i]].view(np.uint32), wdx[i, :ln[i]].view(np.uint32)), i
        assert np.array_equal(col[i, :ln[i]].view(np.uint32), wcol[i, :ln[i]].view(np.uint32)), i


@pytest.mark.parametrize('scene,depth,transparent,bg', [('cube', 1, False, 0), ('cube', 5, True, 0x80FFFFFF),
                                                        ('small', 3, False, 0xFF000000), ('small', 10, True, 0)])
def test_render_parity(cuda, cube_geometry, small_detector, scene, depth, transparent, bg):
    from chroma import gpu
    from chroma.gpu import gpuarray as ga
    from chroma.gpu.packing import PackedGeometry
    geo = cube_geometry if scene == 'cube' else small_detector
    look = (0.0, 0.0, 0.0)
    pos, d = camera_rays(96, 64, (2500.0, -3000.0, 1200.0) if scene == 'cube' else (1800.0, -2400.0, 700.0), look)
    colors = _colors(geo, transparent)
    saved = geo.colors
    geo.colors = colors
    try:
        gg = gpu.GPUGeometry(geo)
        gg.colors    # uploaded now, from these colours
    finally:
        geo.colors = saved
    rays = gpu.GPURays(pos, d, max_alpha_depth=10)
    pix = ga.empty(len(pos), np.uint32)
    rays.render(gg, pix, alpha_depth=depth, bg_color=bg)
    want = oracle.render(PackedGeometry(geo), pos, d, colors, depth, bg_color=bg)
    assert (want[2] > 0).any()
    _compare(rays, pix, want, depth)
    # keep_last_render: rotate the rays about the scene and merge a second render
    axis = np.array([0.0, 0.0, 1.0], np.float32)
    rays.rotate_around_point(0.05, axis, look)
    rays.render(gg, pix, alpha_depth=depth, keep_last_render=True, bg_color=bg)
    pos2 = oracle.transform(pos, 2, phi=0.05, axis=axis, v=look)
    d2 = oracle.transform(d, 1, phi=0.05, axis=axis)
    assert np.array_equal(rays.pos.get().view(np.float32).reshape(-1, 3), pos2)
    assert np.array_equal(rays.dir.get().view(np.float32).reshape(-1, 3), d2)
    _, dx0, len0, col0 = want
    want2 = oracle.render(PackedGeometry(geo), pos2, d2, colors, depth, dx=dx0.copy(), dxlen=len0.copy(),
                          color=col0.copy(), bg_color=bg)
    _compare(rays, pix, want2, depth)


def test_snapshot_and_transforms(cuda, cube_geometry):
    from chroma import gpu
    pos, d = camera_rays(64, 48, (2500.0, -3000.0, 1200.0), (0.0, 0.0, 0.0))
    gg = gpu.GPUGeometry(cube_geometry)
    rays = gpu.GPURays(pos, d)
    colors = np.asarray(cube_geometry.colors, np.uint32)
    from chroma.gpu.packing import PackedGeometry
    snap = rays.snapshot(gg, alpha_depth=4)
    assert np.array_equal(snap, oracle.render(PackedGeometry(cube_geometry), pos, d, colors, 4)[0])
    rays.translate((10.0, -5.0, 2.5))
    rays.rotate(0.3, (0.0, 0.6, 0.8))
    want_pos = oracle.transform(oracle.transform(pos, 0, v=(10.0, -5.0, 2.5)), 1, phi=0.3, axis=(0.0, 0.6, 0.8))
    want_dir = oracle.transform(d, 1, phi=0.3, axis=(0.0, 0.6, 0.8))
    assert np.array_equal(rays.pos.get().view(np.float32).reshape(-1, 3), want_pos)
    assert np.array_equal(rays.dir.get().view(np.float32).reshape(-1, 3), want_dir)


def test_hybrid_render_passes(cuda, small_detector, small_packed):
    """camera.py's hybrid loop, one wavelength: update_xyz_lookup over every
    triangle from a light position, then update_xyz_image and process_image."""
    from chroma import gpu
    from chroma.gpu import gpuarray as ga
    from chroma.gpu import render
    gg = gpu.GPUGeometry(small_detector)
    ntri = len(small_packed.triangles)
    nslots = 4096
    rng = gpu.get_rng_states(nslots, seed=11)
    host_rng = oracle.rng_init(nslots, seed=11)
    light, xyz, wl, max_steps = (0.0, 0.0, 0.0), (0.9, 0.8, 0.7), 440.0, 10
    lk1, lk2 = ga.zeros(3 * ntri, np.float32), ga.zeros(3 * ntri, np.float32)
    h1, h2 = np.zeros(3 * ntri, np.float32), np.zeros(3 * ntri, np.float32)
    for offset in range(0, ntri, nslots):
        render.update_xyz_lookup(gg, nslots, ntri, offset, light, rng, wl, xyz, lk1, lk2, max_steps)
        oracle.hybrid_update_xyz_lookup(small_packed, nslots, ntri, offset, light, host_rng, nslots, wl, xyz, h1, h2,
                                        max_steps)
    assert np.array_equal(rng.get().reshape(-1), host_rng), 'RNG states differ after the lookup pass'
    g1, g2 = lk1.get(), lk2.get()
    assert (h1 != 0).any() or (h2 != 0).any(), 'no diffuse reflection reached the lookup'
    for g, h in ((g1, h1), (g2, h2)):
        assert np.array_equal(g != 0, h != 0)
        assert np.allclose(g, h, rtol=1e-5, atol=0)
    # image pass from the oracle's lookup on both sides (bit-exact)
    lk1.set(h1)
    lk2.set(h2)
    pos, d = camera_rays(64, 64, (1800.0, -2400.0, 700.0), (0.0, 0.0, 0.0))
    rays = gpu.GPURays(pos, d)
    img = ga.zeros(3 * len(pos), np.float32)
    himg = np.zeros(3 * len(pos), np.float32)
    rng2 = gpu.get_rng_states(len(pos), seed=12)
    hrng2 = oracle.rng_init(len(pos), seed=12)
    render.update_xyz_image(gg, rays, rng2, wl, xyz, lk1, lk2, img, 3, max_steps)
    oracle.hybrid_update_xyz_image(small_packed, pos, d, hrng2, len(pos), wl, xyz, h1, h2, himg, 3, max_steps)
    assert np.array_equal(img.get().view(np.uint32), himg.view(np.uint32))
    assert np.array_equal(rng2.get().reshape(-1), hrng2)
    pix = ga.empty(len(pos), np.uint32)
    render.process_image(img, pix, 2)
    assert np.array_equal(pix.get(), oracle.hybrid_process_image(himg, 2))
