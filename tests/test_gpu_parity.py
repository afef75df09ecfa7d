"""Parity of the HIP path (through the C ABI) against the CPU oracle.

Contract (BASELINE north star): history flags, last-hit triangles and channel
ids bit-exact; position / direction / polarisation / time / wavelength /
weight within 1e-5 relative.  Both sides use the same portable math and RNG,
so in practice every word matches; the float check below enforces the 1e-5
contract and separately reports the exact-match fraction.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

FLOAT_RTOL = 1e-5


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from chroma.gpu import create_cuda_context
    return create_cuda_context()


def _compare(host, gpu_photons, label):
    got = gpu_photons.get()
    assert np.array_equal(got.flags, host.flags), label + ': flags differ'
    assert np.array_equal(got.last_hit_triangles, host.last_hit_triangles), label + ': last_hit differ'
    exact = 0
    total = 0
    for f in ('pos', 'dir', 'pol', 'wavelengths', 't', 'weights'):
        a = getattr(got, f).astype(np.float64)
        b = getattr(host, f).astype(np.float64)
        both_nan = np.isnan(a) & np.isnan(b)
        scale = np.maximum(np.abs(b), 1.0 if f in ('pos', 'dir', 'pol') else 1e-30)
        bad = ~both_nan & ~(np.abs(a - b) <= FLOAT_RTOL * scale)
        assert not bad.any(), '%s: %s differs beyond %g at %s' % (label, f, FLOAT_RTOL, np.flatnonzero(bad.ravel())[:5])
        exact += int((getattr(got, f).view(np.uint32) == getattr(host, f).view(np.uint32)).sum())
        total += getattr(got, f).size
    assert np.array_equal(got.evidx, host.evidx)
    return exact / total


def _run_both(geometry, packed, photons, nslots, ntpb, max_blocks, max_steps, seed=1, use_weights=False,
              scatter_first=0, ncopies=1):
    from chroma import gpu
    rng = gpu.get_rng_states(nslots, seed=seed)
    gg = gpu.GPUGeometry(geometry)
    gp = gpu.GPUPhotons(photons, ncopies=ncopies)
    gp.propagate(gg, rng, nthreads_per_block=ntpb, max_blocks=max_blocks, max_steps=max_steps,
                 use_weights=use_weights, scatter_first=scatter_first)
    host = oracle.HostPhotons(photons)
    if ncopies > 1:
        for f in host.FIELDS:
            setattr(host, f, np.concatenate([getattr(host, f)] * ncopies))
    st = oracle.rng_init(nslots, seed=seed)
    stats = oracle.propagate(packed, host, st, nslots, ntpb, max_blocks, max_steps, use_weights=use_weights,
                             scatter_first=scatter_first, ncopies=ncopies)
    return gp, host, rng, st, stats


def test_rng_init_parity(cuda):
    from chroma import gpu
    for seed in (1, 2 ** 40 + 12345):
        r = gpu.get_rng_states(100003, seed=seed)
        assert np.array_equal(r.get().reshape(-1), oracle.rng_init(100003, seed=seed))


def test_distance_to_mesh_kat(cuda, cube_geometry):
    """GPU traversal on the reference's ray-intersection KAT == oracle, bit for bit."""
    import ctypes
    from chroma.gpu import GPUGeometry, _native, gpuarray as ga
    from chroma.gpu.tools import current_stream
    from chroma.gpu.packing import PackedGeometry
    from film import film_rays
    pos, d = film_rays()
    gg = GPUGeometry(cube_geometry)
    o = ga.to_gpu(pos.astype(np.float32).reshape(-1))
    dd = ga.to_gpu(d.astype(np.float32).reshape(-1))
    out = ga.zeros(len(pos), np.float32)
    _native.call('chr_distance_to_mesh', ctypes.c_void_p(gg.gpudata), len(pos), o.gpudata, dd.gpudata, out.gpudata,
                 current_stream())
    ref, tri, _ = oracle.distance_to_mesh(PackedGeometry(cube_geometry), pos, d)
    assert np.array_equal(out.get(), ref)


def test_propagate_single_launch_parity(cuda, small_detector, small_packed):
    """< nthreads_per_block*128 photons: all steps in one launch, slot = photon."""
    from chroma.photon_source import isotropic
    photons = isotropic(20000, seed=11)
    gp, host, rng, st, stats = _run_both(small_detector, small_packed, photons, 256 * 1024, 256, 1024, 100)
    frac = _compare(host, gp, 'single-launch')
    assert np.array_equal(rng.get().reshape(-1), st), 'RNG slot states differ after propagate'
    assert frac > 0.999
    assert stats['launches'] == 1


@pytest.mark.parametrize('ntpb,max_blocks,step_launch', [(64, 64, '1'), (64, 64, '0'), (100, 41, '1')])
def test_propagate_multi_launch_parity(cuda, small_detector, small_packed, monkeypatch, ntpb, max_blocks,
                                       step_launch):
    """Per-step relaunch + survivor compaction + chunks sharing RNG slots.
    (64, 64, '1'): one launch per step, work-item = slot looping over the
    step's chunks; '0': the reference's one launch per chunk; (100, 41): a
    slot count that is not a multiple of 64 (per-chunk launches)."""
    from chroma.photon_source import isotropic
    monkeypatch.setenv('CHR_STEP_LAUNCH', step_launch)
    photons = isotropic(30000, seed=12)
    gp, host, rng, st, stats = _run_both(small_detector, small_packed, photons, ntpb * max_blocks, ntpb, max_blocks,
                                         1000)
    _compare(host, gp, 'multi-launch %s' % ((ntpb, max_blocks, step_launch),))
    assert np.array_equal(rng.get().reshape(-1), st)
    assert stats['host_steps'] > 1 and stats['launches'] > stats['host_steps']
    fused = step_launch == '1' and (ntpb * max_blocks) % 64 == 0
    assert (gp.last_stats.launches == gp.last_stats.steps_run) == fused


@pytest.mark.parametrize('use_weights,scatter_first', [(False, 0), (True, 0), (False, 1), (False, -1)])
def test_physics_scene_parity(cuda, use_weights, scatter_first):
    """Every surface model, bulk re-emission, Rayleigh, wire planes."""
    import scenes
    from chroma import loader
    from chroma.gpu.packing import PackedGeometry
    geo = loader.create_geometry_from_obj(scenes.physics_scene())
    packed = PackedGeometry(geo)
    photons = scenes.photon_sources(24000, seed=21)
    gp, host, rng, st, stats = _run_both(geo, packed, photons, 128 * 256, 128, 256, 60, seed=3,
                                         use_weights=use_weights, scatter_first=scatter_first)
    _compare(host, gp, 'scene w=%s sf=%s' % (use_weights, scatter_first))
    assert np.array_equal(rng.get().reshape(-1), st)
    if not use_weights and scatter_first == 0:     # use_weights disables bulk absorption
        fl = host.flags
        for bit in (1 << 1, 1 << 3, 1 << 4, 1 << 5, 1 << 6, 1 << 7, 1 << 8, 1 << 9):
            assert ((fl & bit) != 0).any(), 'branch bit %d never exercised' % bit
        assert (host.last_hit_triangles == -2).any(), 'wire planes never hit'


def test_ncopies_and_selection_parity(cuda, small_detector, small_packed):
    from chroma import gpu
    from chroma.photon_source import isotropic
    photons = isotropic(5000, seed=13)
    gp, host, rng, st, _ = _run_both(small_detector, small_packed, photons, 64 * 128, 64, 128, 50, ncopies=3)
    _compare(host, gp, 'ncopies')
    det = gpu.GPUDetector(small_detector)
    hits = gp.get_flat_hits(det)
    idx, ch = oracle.hits(host, small_detector.solid_id, small_detector.solid_id_to_channel_index)
    assert np.array_equal(hits.channel.astype(np.int64), ch.astype(np.int64))
    assert np.array_equal(hits.last_hit_triangles, host.last_hit_triangles[idx])
    assert np.array_equal(hits.t, host.t[idx])
    sel = gp.select(1 << 3).get()
    assert np.array_equal(sel.flags, host.flags[oracle.select(host, 1 << 3)])
    copies = list(gp.iterate_copies())
    assert len(copies) == 3 and len(copies[1]) == 5000
    q = gpu.gpuarray.to_gpu(np.arange(len(gp), dtype=np.uint32)[::-1].copy())
    rev = gp.copy_queue(q, len(gp)).get()
    assert np.array_equal(rev.flags, host.flags[::-1])


def test_simulation_end_to_end(cuda, small_detector, small_packed):
    """Simulation.simulate: batching, evidx, per-event hit split."""
    from chroma.sim import Simulation
    from chroma.photon_source import isotropic
    from chroma.event import Photons
    sim = Simulation(small_detector, seed=7, nthreads_per_block=64, max_blocks=256)
    events = [isotropic(3000, seed=30 + i) for i in range(3)]
    out = list(sim.simulate(events, keep_photons_end=True, max_steps=200))
    assert len(out) == 3
    joined = Photons.join(events)
    joined.evidx[:] = np.repeat(np.arange(3), 3000)
    host = oracle.HostPhotons(joined)
    host.last_hit_triangles[:] = -1
    host.weights[:] = 1.0
    st = oracle.rng_init(64 * 256, seed=7)
    oracle.propagate(small_packed, host, st, 64 * 256, 64, 256, 200)
    for i, ev in enumerate(out):
        sl = slice(3000 * i, 3000 * (i + 1))
        assert np.array_equal(ev.photons_end.flags, host.flags[sl])
        idx, ch = oracle.hits(host, small_detector.solid_id, small_detector.solid_id_to_channel_index)
        mine = idx[(idx >= 3000 * i) & (idx < 3000 * (i + 1))]
        assert len(ev.flat_hits) == len(mine)
        assert sum(len(v) for v in ev.hits.values()) == len(mine)


def test_scintillator_detector_parity(cuda):
    """BASELINE config 5 geometry (chroma.demo.scint.tiny(): liquid scintillator
    with 2-component bulk re-emission, light cones cycling shiny / dichroic /
    WLS): HIP == oracle, hits included, with the re-emission branches taken."""
    from chroma import gpu, loader
    from chroma.demo import scint
    from chroma.gpu.packing import PackedGeometry
    from chroma.photon_source import isotropic
    geo = loader.create_geometry_from_obj(scint.tiny())
    packed = PackedGeometry(geo)
    photons = isotropic(30000, seed=5)
    gp, host, rng, st, _ = _run_both(geo, packed, photons, 128 * 256, 128, 256, 1000, seed=9)
    _compare(host, gp, 'scint')
    assert np.array_equal(rng.get().reshape(-1), st)
    fl = host.flags
    for bit in (1 << 7, 1 << 9, 1 << 2):            # SURFACE_REEMIT, BULK_REEMIT, SURFACE_DETECT
        assert ((fl & bit) != 0).any(), 'branch bit %d never exercised' % bit
    hits = gp.get_flat_hits(gpu.GPUDetector(geo))
    idx, ch = oracle.hits(host, geo.solid_id, geo.solid_id_to_channel_index)
    assert np.array_equal(hits.channel.astype(np.int64), ch.astype(np.int64))


def test_scintillator_physics_tables_fit_lds(cuda):
    """The scintillator geometry's hot physics tables (identical tables stored
    once; the components' wavelength tables included) fit the tail kernel's
    LDS copy (propagate.hip TAIL_PHYS_WORDS = 8192 words); the 20,000-entry
    time CDFs and their bucket indexes stay in HBM."""
    from chroma import gpu, loader
    from chroma.demo import scint
    geo = loader.create_geometry_from_obj(scint.tiny())
    hot, total = gpu.GPUGeometry(geo).phys_words()
    assert hot <= 8192, hot
    assert total - hot >= 2 * 20000, (hot, total)
