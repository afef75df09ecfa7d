"""The reference's own tests of the propagation path, run on the HIP path:
test/test_propagation.py (normal-incidence abort), test/test_rayleigh.py
(Rayleigh angular distribution; the ROOT fit replaced by KS and chi-square tests
against the same (1 + cos^2) sin shape with scipy) and
test/test_gpu_photon_gpu_input.py (GPU-resident photon inputs).  Reference
arguments that its current Simulation no longer accepts (geant4_processes)
are dropped.  test_gpu_photon_gpu_input's test_alias_when_single_copy expects
GPUPhotons to alias GPU inputs, but the reference's GPUPhotons copies them
(photon.py:66-82 memcpy_dtod); this build copies as the implementation does."""
from types import SimpleNamespace
from unittest import mock

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from chroma.gpu import create_cuda_context
    return create_cuda_context()


def _axis_photons(n, seed=0, pol=None):
    from chroma.event import Photons
    rng = np.random.default_rng(seed)
    pos = np.tile([0, 0, 0], (n, 1)).astype(np.float32)
    dir = np.tile([0, 0, 1], (n, 1)).astype(np.float32)
    p = np.zeros_like(pos)
    if pol is None:
        phi = rng.uniform(0, 2 * np.pi, n).astype(np.float32)
        p[:, 0] = np.cos(phi)
        p[:, 1] = np.sin(phi)
    else:
        p[:] = pol
    return Photons(pos=pos, dir=dir, pol=p, t=np.zeros(n, np.float32), wavelengths=np.full(n, 400.0, np.float32))


def test_abort_at_normal_incidence(cuda):
    """test_propagation.py:12-56: axis-aligned photons hitting a box face at
    exactly normal incidence neither produce NaNs nor abort."""
    from chroma.geometry import Solid, Geometry, vacuum
    from chroma.loader import create_geometry_from_obj
    from chroma.make import box
    from chroma.sim import Simulation
    cube = Geometry(vacuum)
    cube.add_solid(Solid(box(100, 100, 100), vacuum, vacuum))
    geo = create_geometry_from_obj(cube, update_bvh_cache=False)
    sim = Simulation(geo, seed=5)
    photons = _axis_photons(10000)
    end = next(sim.simulate([photons], keep_photons_end=True, max_steps=1)).photons_end
    for f in ('pos', 'dir', 'pol', 't', 'wavelengths'):
        assert not np.isnan(getattr(end, f)).any(), f
    end = next(sim.simulate([photons], keep_photons_end=True, max_steps=10)).photons_end
    aborted = (end.flags & (1 << 15)) > 0          # NAN_ABORT is bit 15 on the device (photon.h:29,67)
    assert not aborted.any()


@pytest.mark.parametrize('half_size', [50.0, 50000.0])
def test_rayleigh_angular_distribution(cuda, half_size):
    """test_rayleigh.py:33-54: fully polarised photons in water scatter with
    the (1 + cos^2 theta) sin theta distribution.  The reference's 100 mm cube
    gives a few dozen scatters (KS test); a 100 m cube gives tens of thousands
    (KS and chi-square tests)."""
    import scipy.stats
    from chroma.geometry import Solid, Geometry
    from chroma.loader import create_geometry_from_obj
    from chroma.make import box
    from chroma.sim import Simulation
    from chroma.demo.optics import water
    cube = Geometry(water)
    cube.add_solid(Solid(box(2 * half_size, 2 * half_size, 2 * half_size), water, water))
    geo = create_geometry_from_obj(cube, update_bvh_cache=False)
    sim = Simulation(geo, seed=11)
    photons = _axis_photons(100000, pol=[1.0, 0.0, 0.0])
    end = next(sim.simulate([photons], keep_photons_end=True, max_steps=1)).photons_end
    assert not ((end.flags & (1 << 15)) > 0).any()
    scattered = (end.flags & (1 << 4)) > 0
    assert scattered.sum() > 20
    cos_t = np.clip((photons.dir[scattered] * end.dir[scattered]).sum(axis=1).astype(np.float64), -1.0, 1.0)
    theta = np.arccos(cos_t)

    def F(t):   # antiderivative of (1 + cos^2 t) sin t
        return -np.cos(t) - np.cos(t) ** 3 / 3.0

    def cdf(t):
        return (F(t) - F(0.0)) / (F(np.pi) - F(0.0))
    assert scipy.stats.kstest(theta, cdf).pvalue > 1e-3
    if scattered.sum() > 5000:
        edges = np.linspace(0, np.pi, 41)
        hist, _ = np.histogram(theta, bins=edges)
        expected = np.diff(cdf(edges)) * hist.sum()
        assert scipy.stats.chisquare(hist, expected).pvalue > 1e-3


def _gpu_view(gp):
    return SimpleNamespace(pos=gp.pos, dir=gp.dir, pol=gp.pol, wavelengths=gp.wavelengths, t=gp.t,
                           last_hit_triangles=gp.last_hit_triangles, flags=gp.flags, weights=gp.weights,
                           evidx=gp.evidx)


def _two_photons():
    from chroma import event
    return event.Photons(np.array([[0, 0, 0], [1, 2, 3]], np.float32), np.array([[1, 0, 0], [0, 1, 0]], np.float32),
                         np.array([[0, 1, 0], [0, 0, 1]], np.float32), np.array([400.0, 420.0], np.float32),
                         np.array([0.1, 0.2], np.float32), flags=np.array([0, 1], np.uint32),
                         weights=np.array([1.0, 0.5], np.float32), evidx=np.array([0, 0], np.uint32))


def test_gpu_input_copies_duplicates_and_resets(cuda):
    """test_gpu_photon_gpu_input.py:52-83: GPUPhotons from GPU arrays (copied
    device to device), replicated with ncopies, and with the optional fields
    reset."""
    from chroma import gpu
    src = gpu.GPUPhotons(_two_photons())
    same = gpu.GPUPhotons(_gpu_view(src))
    assert same.true_nphotons == 2
    assert np.array_equal(same.pos.get(), src.pos.get()) and np.array_equal(same.flags.get(), src.flags.get())
    dup = gpu.GPUPhotons(_gpu_view(src), ncopies=2)
    assert len(dup.pos) == 4
    pos = dup.pos.get().view(np.float32).reshape(-1, 3)
    np.testing.assert_allclose(pos[:2], pos[2:])
    fl = dup.flags.get()
    assert np.array_equal(fl[:2], fl[2:])
    reset = gpu.GPUPhotons(_gpu_view(src), copy_flags=False, copy_triangles=False, copy_weights=False)
    assert int(reset.flags.gpudata) != int(src.flags.gpudata)
    assert (reset.flags.get() == 0).all() and (reset.last_hit_triangles.get() == -1).all()
    assert np.allclose(reset.weights.get(), 1.0)


def test_simulate_accepts_gpu_photons(cuda):
    """test_gpu_photon_gpu_input.py:85-106: Simulation joins GPU-resident
    sources on the device (no CPU Photons.join)."""
    import chroma.demo
    from chroma import event, gpu
    from chroma.loader import create_geometry_from_obj
    from chroma.sim import Simulation
    det = create_geometry_from_obj(chroma.demo.tiny(), update_bvh_cache=False)
    sim = Simulation(det, seed=3)
    one = event.Photons(np.array([[0.0, 0.0, 0.0]], np.float32), np.array([[0.0, 0.0, 1.0]], np.float32),
                        np.array([[1.0, 0.0, 0.0]], np.float32), np.array([400.0], np.float32),
                        np.array([0.0], np.float32))
    ev = event.Event(photons_beg=gpu.GPUPhotons(one))
    with mock.patch('chroma.event.Photons.join', side_effect=AssertionError('CPU join used for GPU sources')):
        results = list(sim.simulate([ev], keep_hits=False, keep_flat_hits=False, run_daq=False, max_steps=1))
    assert len(results) == 1
