"""HIP DAQ (csrc/daq.hip through the C ABI) against the CPU oracle, bit for
bit, and the reference's own DAQ test (test/test_detector.py) through
Simulation(run_daq=True)."""
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


@pytest.mark.parametrize('ndaq,ntpb,max_blocks,charge', [
    (1, 64, 8, (1.0, 0.1, 0.5, 1.5)), (1, 256, 1024, (1.0, 0.1, 0.5, 1.5)), (5, 64, 16, (1.0, 0.1, 0.5, 1.5)),
    # a pedestal-like charge CDF with negative support: negative charges convert
    # to 0 (CUDA's saturating float -> u32; a plain cast is undefined)
    (1, 64, 8, (0.1, 0.5, -2.0, 2.0)), (5, 64, 16, (0.1, 0.5, -2.0, 2.0))])
def test_daq_parity(cuda, small_detector, small_packed, ndaq, ntpb, max_blocks, charge):
    from chroma import gpu
    from chroma.gpu.detector import cdf_arrays
    from chroma.photon_source import isotropic
    from test_gpu_parity import _run_both, _compare
    saved = small_detector.time_cdf, small_detector.charge_cdf
    small_detector.set_time_dist_gaussian(1.2, -6.0, 6.0)
    small_detector.set_charge_dist_gaussian(*charge)
    try:
        photons = isotropic(20000, seed=31)
        nslots = 64 * 1024
        gp, host, rng, st, _ = _run_both(small_detector, small_packed, photons, nslots, 64, 1024, 100, seed=5)
        _compare(host, gp, 'propagate before DAQ')
        gdet = gpu.GPUDetector(small_detector)
        daq = gpu.GPUDaq(gdet, ndaq=ndaq)
        normal = np.zeros(2 * nslots, np.uint32)
        for start, n in ((0, 7000), (7000, 13000)):     # two "events"
            daq.begin_acquire()
            daq.acquire(gp, rng, nthreads_per_block=ntpb, max_blocks=max_blocks, start_photon=start, nphotons=n)
            ch = daq.end_acquire().get()
            t, q, fl = oracle.daq(host, small_detector.solid_id, small_detector.solid_id_to_channel_index,
                                  cdf_arrays(small_detector.time_cdf), cdf_arrays(small_detector.charge_cdf),
                                  gdet.charge_unit, st, nslots, normal_cache=normal, start=start, n=n, ndaq=ndaq,
                                  nchannels=gdet.nchannels, nthreads_per_block=ntpb, max_blocks=max_blocks)
            assert ch.hit.sum() > 0
            assert np.array_equal(ch.t.view(np.uint32), t.view(np.uint32)), 'earliest times differ'
            assert np.array_equal(ch.q.view(np.uint32), q.view(np.uint32)), 'charges differ'
            assert np.array_equal(ch.flags, fl), 'channel histories differ'
            assert np.array_equal(rng.get().reshape(-1), st), 'RNG slot states differ after DAQ'
            if ndaq > 1:
                assert np.array_equal(rng.normal_cache.get(), normal)
    finally:
        small_detector.time_cdf, small_detector.charge_cdf = saved


def _box_sim():
    from chroma.detector import Detector
    from chroma.geometry import Solid, vacuum
    from chroma.loader import create_geometry_from_obj
    from chroma.make import box
    from chroma.demo.optics import r7081hqe_photocathode
    from chroma.sim import Simulation
    cube = Detector(vacuum)
    cube.add_pmt(Solid(box(10.0, 10, 10), vacuum, vacuum, surface=r7081hqe_photocathode))
    cube.set_time_dist_gaussian(1.2, -6.0, 6.0)
    cube.set_charge_dist_gaussian(1.0, 0.1, 0.5, 1.5)
    geo = create_geometry_from_obj(cube, update_bvh_cache=False)
    return Simulation(geo, seed=17)


def _one_photon(t0):
    from chroma.event import Photons
    pos = np.zeros((1, 3), np.float32)
    dir = np.tile([0, 0, 1], (1, 1)).astype(np.float32)
    phi = np.random.uniform(0, 2 * np.pi, 1).astype(np.float32)
    pol = np.zeros_like(pos)
    pol[:, 0], pol[:, 1] = np.cos(phi), np.sin(phi)
    return Photons(pos=pos, dir=dir, pol=pol, t=np.full(1, t0, np.float32), wavelengths=np.full(1, 400.0, np.float32))


def test_detector_time_and_charge(cuda):
    """test/test_detector.py testTime / testCharge, unmodified in substance."""
    sim = _box_sim()
    hit_times = [ev.channels.t[0] for ev in sim.simulate((_one_photon(100.0) for _ in range(1000)), run_daq=True)
                 if ev.channels.hit[0]]
    assert len(hit_times) > 100
    assert abs(np.std(hit_times) - 1.2) < 0.1
    hit_q = [ev.channels.q[0] for ev in sim.simulate((_one_photon(0.0) for _ in range(1000)), run_daq=True)
             if ev.channels.hit[0]]
    assert abs(np.mean(hit_q) - 1.0) < 0.1
    assert abs(np.std(hit_q) - 0.1) < 0.1
