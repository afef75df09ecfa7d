"""HIP PDF kernels (csrc/pdf.hip through GPUPDF / GPUKernelPDF and the C
ABI) against the CPU oracle bit for bit, and the reference's own PDF test
(test/test_pdf.py testGPUPDF: propagate -> DAQ -> add_hits_to_pdf, then
hitcount > 0, pdf > 0 and hitcount[c] == pdf[c].sum()) with an isotropic
source in place of the Geant4 generator (absent here)."""
from types import SimpleNamespace

import numpy as np
import pytest

import oracle
from test_pdf import _channels

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from chroma.gpu import create_cuda_context
    return create_cuda_context()


def _gpu_channels(t, q, ndaq=1):
    from chroma.gpu import gpuarray as ga
    return SimpleNamespace(t=ga.to_gpu(t), q=ga.to_gpu(q), ndaq=ndaq)


def test_bin_hits_parity(cuda):
    from chroma import gpu
    n, tb, qb, tr, qr = 29007, 100, 10, (-0.5, 99.5), (-0.5, 9.5)
    p = gpu.GPUPDF()
    p.setup_pdf(n, tb, tr, qb, qr)
    p.clear_pdf()
    hc = np.zeros(n, np.uint32)
    pdf = np.zeros(n * tb * qb, np.uint32)
    for ev in range(4):
        t, q = _channels(n, seed=100 + ev)
        p.add_hits_to_pdf(_gpu_channels(t, q))
        oracle.pdf_bin_hits(q, t, hc, pdf, tb, tr, qb, qr)
    ghc, gpdf = p.get_pdfs()
    assert p.events_in_histogram == 4
    assert np.array_equal(ghc, hc)
    assert np.array_equal(gpdf.reshape(-1), pdf)
    assert np.array_equal(ghc, gpdf.reshape(n, -1).sum(axis=1))


@pytest.mark.parametrize('ndaq,k,n,nan', [(1, 10, 2000, False), (64, 10, 2000, False), (300, 50, 2000, False),
                                          (64, 10, 2000, True),        # NaN MC times: defined order (NaN last)
                                          (4200, 4200, 300, False)])   # > 8192 candidates: unstaged branch
def test_pdf_eval_parity(cuda, ndaq, k, n, nan):
    from chroma import gpu
    w, tr = 2.0, (-10.0, 100.0)
    r = np.random.default_rng(ndaq)
    event_hit = (r.random(n) < 0.4).astype(np.uint32)
    event_time = r.uniform(0, 90, n).astype(np.float32)
    p = gpu.GPUPDF()
    p.setup_pdf_eval(event_hit, event_time, np.zeros(n, np.float32), w, tr, 1.0, (0.0, 10.0), min_bin_content=k)
    nhit = int(event_hit.sum())
    hc, bc = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    near = np.full(nhit * k, 1e9, np.float32)
    for ev in range(2):                                  # two MC accumulations
        t, q = _channels(n, ndaq, seed=7 + ev)
        if nan:
            t[r.random(len(t)) < 0.05] = np.nan
        p.accumulate_pdf_eval(_gpu_channels(t, q, ndaq))
        queues = np.ones(nhit * (ndaq + 1), np.uint32)
        oracle.pdf_accumulate_bincount(event_hit, event_time, t, ndaq, hc, bc, queues, w, tr, k,
                                       p.map_channel_id_to_hit_offset)
        oracle.pdf_accumulate_nearest(p.map_hit_offset_to_channel_id, queues, event_time, t, ndaq, near, k)
        assert np.array_equal(p.work_queues.get(), queues)
    assert np.array_equal(p.eval_hitcount_gpu.get(), hc)
    assert np.array_equal(p.eval_bincount_gpu.get(), bc)
    assert np.array_equal(p.nearest_mc_gpu.get().view(np.uint32), near.view(np.uint32))
    hitcount, value, uncert = p.get_pdf_eval()
    assert np.array_equal(hitcount, hc) and (value > 0).any()
    if not nan:
        assert np.all(np.isfinite(value))


@pytest.mark.parametrize('time_only', [True, False])
def test_kernel_pdf_parity(cuda, time_only):
    from chroma import gpu
    n, tr, qr = 29007, (-10.0, 100.0), (0.0, 10.0)
    r = np.random.default_rng(2)
    eh = (r.random(n) < 0.7).astype(np.uint32)
    et, eq = r.uniform(0, 90, n).astype(np.float32), r.uniform(0, 9, n).astype(np.float32)
    k = gpu.GPUKernelPDF()
    k.setup_moments(n, tr, qr, time_only=time_only)
    mom = [np.zeros(n, np.uint32)] + [np.zeros(n, np.float32) for _ in range(4)]
    for ev in range(3):
        t, q = _channels(n, seed=40 + ev, hit_frac=0.8)
        k.accumulate_moments(_gpu_channels(t, q))
        oracle.pdf_accumulate_moments(time_only, t, q, tr, qr, *mom)
    got = [k.hitcount_gpu, k.tmom1_gpu, k.tmom2_gpu, k.qmom1_gpu, k.qmom2_gpu]
    for g, e in zip(got, mom):
        assert np.array_equal(g.get().view(np.uint32), e.view(np.uint32))
    k.compute_bandwidth(eh, et, eq)
    k.setup_kernel(eh, et, eq)
    hc, tp, qp = np.zeros(n, np.uint32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    itb, iqb = k.inv_time_bandwidths_gpu.get(), k.inv_charge_bandwidths_gpu.get()
    for ev in range(3):
        t, q = _channels(n, seed=60 + ev, hit_frac=0.8)
        k.accumulate_kernel(_gpu_channels(t, q))
        oracle.pdf_accumulate_kernel_eval(time_only, eh, et, eq, t, q, tr, qr, itb, iqb, hc, tp, qp)
    assert np.array_equal(k.hitcount_gpu.get(), hc)
    assert np.array_equal(k.time_pdf_values_gpu.get().view(np.uint32), tp.view(np.uint32))
    assert np.array_equal(k.charge_pdf_values_gpu.get().view(np.uint32), qp.view(np.uint32))
    with np.errstate(invalid='ignore'):
        hitcount, values, _ = k.get_kernel_eval()
    assert np.array_equal(hitcount, hc) and (values > 0).any()
    # NaN values are the reference formula's own (time_pdf * charge_pdf,
    # pdf.py:161-175): a NaN inverse charge bandwidth (its variance is not
    # clipped at 0, pdf.py:99-110) or an infinite kernel sum times a zero one.
    # The oracle has them bit for bit (above); none comes from finite factors.
    with np.errstate(invalid='ignore', divide='ignore'):
        norm = np.maximum(1, hc)
        tpn, qpn = tp / norm, qp / norm
    if not time_only:
        assert not np.isnan(values[np.isfinite(tpn) & np.isfinite(qpn)]).any()


def test_pdf_from_propagate_and_daq(cuda, small_detector):
    """test/test_pdf.py testGPUPDF with an isotropic source (20 events)."""
    from chroma import gpu
    from chroma.photon_source import isotropic
    saved = small_detector.time_cdf, small_detector.charge_cdf
    small_detector.set_time_dist_gaussian(1.2, -6.0, 6.0)
    small_detector.set_charge_dist_gaussian(1.0, 0.1, 0.5, 1.5)
    try:
        gdet = gpu.GPUDetector(small_detector)
    finally:
        small_detector.time_cdf, small_detector.charge_cdf = saved
    nthreads_per_block, max_blocks = 64, 1024
    rng = gpu.get_rng_states(nthreads_per_block * max_blocks)
    daq = gpu.GPUDaq(gdet)
    p = gpu.GPUPDF()
    p.setup_pdf(gdet.nchannels, 100, (-0.5, 999.5), 10, (-0.5, 9.5))
    p.clear_pdf()
    detected = channel_hits = 0
    for ev in range(20):     # a few hundred photons per event: channel charges of a few p.e. (qrange 0-9.5)
        gp = gpu.GPUPhotons(isotropic(400, seed=ev))
        gp.propagate(gdet, rng, nthreads_per_block, max_blocks, max_steps=100)
        detected += int(((gp.flags.get() & 4) != 0).sum())
        daq.begin_acquire()
        daq.acquire(gp, rng, nthreads_per_block, max_blocks)
        ch = daq.end_acquire()
        c = ch.get()
        channel_hits += int(c.hit.sum())
        seen = (c.t[c.hit], c.q[c.hit], len(ch.t), gdet.nchannels)
        p.add_hits_to_pdf(ch)
    assert detected > 0 and channel_hits > 0, (detected, channel_hits)
    hitcount, pdf = p.get_pdfs()
    assert (hitcount > 0).any() and (pdf > 0).any(), (channel_hits, hitcount.sum(), seen)
    for i, nhits in enumerate(hitcount):
        assert nhits == pdf[i].sum()
