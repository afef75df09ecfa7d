"""DAQ (reference chroma/cuda/daq.cu + chroma/gpu/daq.py): the CPU oracle's
statistics against the reference's own test (test/test_detector.py: one
photon per event into a box PMT, time CDF gaussian rms 1.2 on [-6, 6],
charge CDF gaussian mean 1.0 rms 0.1 on [0.5, 1.5]; std(t) = 1.2 +- 0.1,
mean(q) = 1.0 +- 0.1, std(q) = 0.1 +- 0.1), plus the host-side CDF tables."""
import numpy as np

import oracle


def _box_detector():
    from chroma.detector import Detector
    from chroma.geometry import Solid, vacuum
    from chroma.make import box
    from chroma.demo.optics import r7081hqe_photocathode
    cube = Detector(vacuum)
    cube.add_pmt(Solid(box(10.0, 10, 10), vacuum, vacuum, surface=r7081hqe_photocathode))
    cube.set_time_dist_gaussian(1.2, -6.0, 6.0)
    cube.set_charge_dist_gaussian(1.0, 0.1, 0.5, 1.5)
    cube.flatten()
    return cube


def _detected(n, t0=100.0):
    """n photons that ended on triangle 0 of the PMT with SURFACE_DETECT."""
    from chroma.event import Photons
    p = Photons(np.zeros((n, 3), np.float32), np.tile([0, 0, 1.0], (n, 1)).astype(np.float32),
                np.tile([1.0, 0, 0], (n, 1)).astype(np.float32), np.full(n, 400.0, np.float32),
                t=np.full(n, t0, np.float32))
    h = oracle.HostPhotons(p)
    h.flags[:] = 0x4
    h.last_hit_triangles[:] = 0
    return h


def _daq_events(det, nevents, ndaq=1, seed=7):
    from chroma.gpu.detector import cdf_arrays
    tcdf, qcdf = cdf_arrays(det.time_cdf), cdf_arrays(det.charge_cdf)
    unit = np.float32(det.charge_cdf[0][-1] / 2 ** 16)
    nslots = 64 * 4
    st = oracle.rng_init(nslots, seed=seed)
    normal = np.zeros(2 * nslots, np.uint32)
    h = _detected(nevents)
    ts, qs = [], []
    for e in range(nevents):   # one photon per event, one DAQ per event (sim.py:143-152)
        t, q, fl = oracle.daq(h, det.solid_id, det.solid_id_to_channel_index, tcdf, qcdf, unit, st, nslots,
                              normal_cache=normal, start=e, n=1, ndaq=ndaq, nchannels=det.num_channels(),
                              nthreads_per_block=64, max_blocks=4)
        ts.append(t)
        qs.append(q)
        assert fl[0] == 0x4
    return np.array(ts), np.array(qs)


def test_cdf_tables_pad_reference_quirk():
    """Detector._pdf_to_cdf yields one fewer y than x (reference detector.py:101-102);
    the device tables repeat the last y so interp never reads past the end."""
    from chroma.gpu.detector import cdf_arrays
    det = _box_detector()
    x, y = det.time_cdf
    assert len(y) == len(x) - 1 and abs(y[-1] - 1.0) < 1e-12
    dx, dy = cdf_arrays(det.time_cdf)
    assert len(dx) == len(dy) == 51 and dy[-1] == dy[-2] == np.float32(1.0)


def test_daq_time_and_charge_statistics():
    det = _box_detector()
    ts, qs = _daq_events(det, 1000)
    hit = ts[:, 0] < 1e8
    assert hit.all()
    assert abs(ts[hit, 0].std() - 1.2) < 0.1            # test_detector.py:52
    assert abs(qs[hit, 0].mean() - 1.0) < 0.1            # test_detector.py:76
    assert abs(qs[hit, 0].std() - 0.1) < 0.1             # test_detector.py:77
    # charge is quantised in units of charge_cdf_x[-1] / 2^16
    unit = np.float32(1.5 / 2 ** 16)
    assert np.allclose(np.round(qs[:, 0] / unit) * unit, qs[:, 0], rtol=0, atol=1e-7)


def test_daq_many_adds_unit_normal_smear():
    """ndaq > 1 (run_daq_many, daq.cu:131): time = t + N(0,1) + time-CDF sample,
    so the spread becomes sqrt(1.2^2 + 1); charges are converted for the first
    copy only (convert_charge_int_to_float covers nchannels words, daq.cu:164-172)."""
    det = _box_detector()
    ts, qs = _daq_events(det, 400, ndaq=8)
    assert ts.shape == (400, 8)
    assert abs(ts.std() - np.hypot(1.2, 1.0)) < 0.12
    assert (qs[:, 1:] == 0).all() and (qs[:, 0] > 0).all()


def test_daq_undetected_photons_leave_channels_empty():
    det = _box_detector()
    from chroma.gpu.detector import cdf_arrays
    h = _detected(10)
    h.flags[:] = 0x8              # SURFACE_ABSORB: not a detection
    st = oracle.rng_init(64, seed=1)
    before = st.copy()
    t, q, fl = oracle.daq(h, det.solid_id, det.solid_id_to_channel_index, cdf_arrays(det.time_cdf),
                          cdf_arrays(det.charge_cdf), 1.5 / 2 ** 16, st, 64, nchannels=1, nthreads_per_block=64,
                          max_blocks=1)
    assert t[0] == np.float32(1e9) and q[0] == 0 and fl[0] == 0
    assert np.array_equal(st, before)       # no draws for undetected photons
