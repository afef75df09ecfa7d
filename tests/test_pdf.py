"""PDF layer (reference chroma/cuda/pdf.cu + chroma/gpu/pdf.py): the CPU
oracle (oracle/pdf_oracle.c) against independent numpy / pure-Python
restatements of each kernel, and the shared erff against math.erf.  No
fixture of the reference pins these kernels (test/test_pdf.py needs Geant4):
the per-channel consistency it asserts (hitcount == pdf[channel].sum()) is
checked here and on the GPU (test_gpu_pdf.py)."""
import math

import numpy as np

import oracle


def _channels(n, ndaq=1, seed=3, hit_frac=0.6):
    r = np.random.default_rng(seed)
    t = r.uniform(-20, 120, n * ndaq).astype(np.float32)
    t[r.random(n * ndaq) > hit_frac] = np.float32(1e9)          # not hit (daq.py maxtime)
    q = r.uniform(-1, 12, n * ndaq).astype(np.float32)
    return t, q


def test_erff_against_math_erf():
    x = np.concatenate([np.linspace(-6, 6, 20001), [0.0, -0.0, 1e-30, 0.4999999, 0.5, 3.9999, 4.0, 50.0]])
    y = oracle.erff(x)
    ref = np.array([math.erf(float(np.float32(v))) for v in x])
    assert np.max(np.abs(y - ref)) < 3e-7      # A&S 7.1.26 (1.5e-7) + float32 rounding
    small = np.abs(x) < 0.5
    nz = small & (x != 0)
    assert np.max(np.abs(y[nz] - ref[nz]) / np.abs(ref[nz])) < 1e-6
    assert y[x == 0.0][0] == 0.0 and np.all(np.abs(y[np.abs(x) >= 4]) == 1.0)


def test_bin_hits_matches_numpy_and_is_consistent():
    n, tb, qb, tr, qr = 500, 100, 10, (-0.5, 99.5), (-0.5, 9.5)
    t, q = _channels(n)
    hitcount = np.zeros(n, np.uint32)
    pdf = np.zeros(n * tb * qb, np.uint32)
    for _ in range(3):                                  # accumulates across events
        oracle.pdf_bin_hits(q, t, hitcount, pdf, tb, tr, qb, qr)
    pdf = pdf.reshape(n, tb, qb)
    # numpy restatement: q through a saturating u32 conversion, float32 bin arithmetic
    qf = np.where(q > 0, np.floor(q), 0).astype(np.float32)
    f32 = np.float32
    sel = (t < f32(1e8)) & (t >= f32(tr[0])) & (t < f32(tr[1])) & (qf >= f32(qr[0])) & (qf < f32(qr[1]))
    tbin = np.minimum(((t - f32(tr[0])) / (f32(tr[1]) - f32(tr[0])) * f32(tb)).astype(np.int64), tb - 1)
    qbin = np.minimum(((qf - f32(qr[0])) / (f32(qr[1]) - f32(qr[0])) * f32(qb)).astype(np.int64), qb - 1)
    exp = np.zeros((n, tb, qb), np.uint32)
    idx = np.flatnonzero(sel)
    exp[idx, tbin[idx], qbin[idx]] = 3
    assert np.array_equal(pdf, exp)
    assert np.array_equal(hitcount, 3 * sel.astype(np.uint32))
    assert np.array_equal(hitcount, pdf.reshape(n, -1).sum(axis=1))     # test_pdf.py:46-47


def _python_pdf_eval(event_hit, event_time, mc, ndaq, k, min_twidth, trange):
    """pure-Python pdf.cu:34-150 (bincount + nearest) for one accumulate call."""
    n = len(event_hit)
    hc = np.zeros(n, np.uint32)
    bc = np.zeros(n, np.uint32)
    nearest = {}
    for c in range(n):
        h, b, d = 0.0, 0.0, []
        for i in range(ndaq):
            v = float(mc[i * n + c])
            if v >= 1e8 or v < trange[0] or v > trange[1]:
                continue
            h += 1
            if not event_hit[c]:
                continue
            dist = abs(np.float32(mc[i * n + c]) - np.float32(event_time[c]))
            if float(dist) < min_twidth / 2.0:
                b += 1
            if b < k:
                d.append(float(dist))
        hc[c], bc[c] = h, b
        if event_hit[c]:
            nearest[c] = sorted(d)[:k]
    return hc, bc, nearest


def test_pdf_eval_bincount_and_nearest_match_python():
    n, ndaq, k, w, tr = 300, 40, 10, 2.0, (-10.0, 100.0)
    t, _ = _channels(n, ndaq, seed=9)
    r = np.random.default_rng(4)
    event_hit = (r.random(n) < 0.5).astype(np.uint32)
    event_time = r.uniform(0, 90, n).astype(np.float32)
    nhit = int(event_hit.sum())
    m_c2h = np.maximum(0, np.cumsum(event_hit) - 1).astype(np.uint32)
    m_h2c = np.flatnonzero(event_hit).astype(np.uint32)
    hc = np.zeros(n, np.uint32)
    bc = np.zeros(n, np.uint32)
    queues = np.ones(nhit * (ndaq + 1), np.uint32)
    near = np.full(nhit * k, 1e9, np.float32)
    oracle.pdf_accumulate_bincount(event_hit, event_time, t, ndaq, hc, bc, queues, w, tr, k, m_c2h)
    oracle.pdf_accumulate_nearest(m_h2c, queues, event_time, t, ndaq, near, k)
    ehc, ebc, enear = _python_pdf_eval(event_hit, event_time, t, ndaq, k, w, tr)
    assert np.array_equal(hc, ehc) and np.array_equal(bc, ebc)
    near = near.reshape(nhit, k)
    for h, c in enumerate(m_h2c):
        got = near[h][near[h] < 1e8]
        assert np.array_equal(got, np.array(enear[c], np.float32)), c


def test_kernel_moments_and_eval_against_numpy():
    n, tr, qr = 400, (-10.0, 100.0), (0.0, 10.0)
    t, q = _channels(n, seed=12, hit_frac=0.8)
    for time_only in (1, 0):
        mom0 = np.zeros(n, np.uint32)
        acc = [np.zeros(n, np.float32) for _ in range(4)]
        oracle.pdf_accumulate_moments(time_only, t, q, tr, qr, mom0, *acc)
        sel = (t >= tr[0]) & (t <= tr[1])
        if not time_only:
            sel &= (q >= qr[0]) & (q <= qr[1])
        assert np.array_equal(mom0, sel.astype(np.uint32))
        assert np.array_equal(acc[0], np.where(sel, t, 0).astype(np.float32))
        assert np.allclose(acc[1], np.where(sel, t.astype(np.float64) ** 2, 0), rtol=1e-6)
        r = np.random.default_rng(5)
        eh = (r.random(n) < 0.7).astype(np.uint32)
        et, eq = r.uniform(0, 90, n).astype(np.float32), r.uniform(0, 9, n).astype(np.float32)
        itb, iqb = r.uniform(0.05, 2, n).astype(np.float32), r.uniform(0.5, 3, n).astype(np.float32)
        itb[:10] = 0.0                                  # zero bandwidth: flat window norm (pdf.cu:313)
        hc = np.zeros(n, np.uint32)
        tp, qp = np.zeros(n, np.float32), np.zeros(n, np.float32)
        oracle.pdf_accumulate_kernel_eval(time_only, eh, et, eq, t, q, tr, qr, itb, iqb, hc, tp, qp)
        assert np.array_equal(hc, sel.astype(np.uint32))
        erf = np.vectorize(math.erf)
        g = sel & (eh != 0)
        tt, ib = t.astype(np.float64), itb.astype(np.float64)
        norm = np.where(ib > 0, (erf((tr[1] - tt) * ib / math.sqrt(2)) - erf((tr[0] - tt) * ib / math.sqrt(2)))
                        * math.sqrt(math.pi / 2), tr[1] - tr[0])
        with np.errstate(divide='ignore', invalid='ignore'):
            term = np.exp(-0.5 * ((tt - et) * ib) ** 2) * (ib if time_only else 1.0) / norm
        exp = np.where(g, term, 0.0)
        assert np.allclose(tp, exp, rtol=2e-5, atol=1e-7)
        if not time_only:
            qq, iq = q.astype(np.float64), iqb.astype(np.float64)
            qnorm = (erf((qr[1] - qq) * iq / math.sqrt(2)) - erf((qr[0] - qq) * iq / math.sqrt(2))) \
                * math.sqrt(math.pi / 2)
            qexp = np.where(g, np.exp(-0.5 * ((qq - eq) * iq) ** 2) / qnorm, 0.0)
            assert np.allclose(qp, qexp, rtol=2e-5, atol=1e-7)
