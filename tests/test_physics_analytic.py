"""The photon physics pinned to closed forms outside the oracle (VERDICT r04
item 2).

HIP == oracle bit for bit is the parity gate elsewhere; these tests tie both
to physics neither of them computes: each scene isolates one process of the
reference (chroma/cuda/photon.h), one step is propagated, and the outcome
frequencies / distributions are compared with the analytic answer.

  * Fresnel at a planar interface (propagate_at_boundary, photon.h:572-632):
    R_s = (sin(ti - tt) / sin(ti + tt))^2, R_p = (tan(ti - tt) / tan(ti + tt))^2,
    ((n1 - n2) / (n1 + n2))^2 near normal incidence, R_p = 0 at Brewster's angle,
    Snell refraction n1 sin ti = n2 sin tt, total internal reflection beyond
    the critical angle, the exact mirror direction of a reflection;
  * Beer-Lambert (propagate_to_boundary, photon.h:455-570): the bulk absorption
    and Rayleigh scattering distances are exponential with the tables' lengths
    (fraction within the boundary distance, KS of the distances), and the time
    advances by distance * n / c;
  * the diffuse reflector (photon.h:648-667) is Lambertian: cos(theta) to the
    normal has CDF cos^2, the azimuth is uniform;
  * the specular reflector (photon.h:634-646) mirrors about the normal;
  * the thin-film COMPLEX surface (photon.h:669-827): R and T are the Airy
    sums of the single absorbing layer (computed here in complex128 from the
    Fresnel amplitudes; the kernel expands them into real arithmetic), and the
    outcome frequencies follow absorb = 1 - R - T, detect | absorb, diffuse | reflect;
  * the WLS surface (photon.h:829-874): re-emitted wavelengths follow the
    surface's reemission CDF (linear between grid points, sample_cdf,
    random.h:34-55), directions are isotropic.

Each test runs on the HIP path (-m gpu) and on the CPU oracle (its own
restatement, so the oracle is pinned every CPU run).  Statistical checks:
binomial / chi-square / KS p-values above 1e-3 at fixed seeds (the photons are
deterministic, and HIP == oracle, so both backends see the same p-values);
geometric ones within float32 tolerances stated at each assert.
"""
import numpy as np
import pytest
import scipy.stats

import oracle

BACKENDS = [pytest.param('hip', marks=pytest.mark.gpu), 'oracle']
# 2^21 RNG slots: every photon of a test draws from its own fresh subsequence.
# (With the reference's slot reuse across chunks the outcome frequencies still
# follow the closed forms to statistical precision on most seeds, but a later
# chunk's draws continue the streams of an earlier one, so they are not the
# independent samples a binomial / chi-square test assumes.)
NTPB, MAXB = 256, 8192
P_MIN = 1e-3
C_MM_NS = 299.792458          # physical_constants.h:5

NOWHERE = 1e20                # an absorption / scattering length that never acts in a 1e4 mm scene


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from chroma.gpu import create_cuda_context
    return create_cuda_context()


def _material(name, n, absl=NOWHERE, scat=NOWHERE):
    from chroma.geometry import Material
    m = Material(name)
    m.set('refractive_index', n)
    m.set('absorption_length', absl)
    m.set('scattering_length', scat)
    return m


def _slab_geometry(inside, outside, surface=None):
    """A 20 m x 20 m x 1 m slab of `inside` in `outside`, top face at z = 0."""
    from chroma import make
    from chroma.geometry import Geometry, Solid
    from chroma.loader import create_geometry_from_obj
    g = Geometry(outside)
    g.add_solid(Solid(make.box(20000.0, 20000.0, 1000.0), inside, outside, surface=surface), displacement=(0, 0, -500))
    return create_geometry_from_obj(g, update_bvh_cache=False)


def _photons(pos, d, pol, wl=400.0):
    from chroma.event import Photons
    d = np.asarray(d, np.float32)
    n = len(d)
    pos = np.broadcast_to(np.asarray(pos, np.float32), (n, 3)).copy()
    return Photons(pos, d, np.asarray(pol, np.float32), np.full(n, wl, np.float32), np.zeros(n, np.float32))


def _propagate(backend, geo, photons, max_steps=1, seed=1, request=None):
    """One propagate of `photons` in `geo`; returns the end photons (numpy fields)."""
    from chroma.gpu.packing import PackedGeometry
    if backend == 'hip':
        request.getfixturevalue('cuda')
        from chroma import gpu
        rng = gpu.get_rng_states(NTPB * MAXB, seed=seed)
        gp = gpu.GPUPhotons(photons, copy_flags=True, copy_triangles=False, copy_weights=False)
        gp.propagate(gpu.GPUGeometry(geo), rng, nthreads_per_block=NTPB, max_blocks=MAXB, max_steps=max_steps)
        return gp.get()
    host = oracle.HostPhotons(photons)
    host.flags[:] = 0
    host.last_hit_triangles[:] = -1
    host.weights[:] = 1
    st = oracle.rng_init(NTPB * MAXB, seed=seed)
    oracle.propagate(PackedGeometry(geo), host, st, NTPB * MAXB, NTPB, MAXB, max_steps)
    return host


def _incidence(theta, n, hit=(37.3, 21.7, 0.0), height=100.0, side=1.0):
    """n photons hitting the plane z = 0 at (hit) with incidence angle theta,
    from z = side*height; the direction has a small y component so that no
    component is exactly zero (a zero component makes a 'flat' walk).
    Returns (start position, direction, s-polarisation, p-polarisation, normal
    facing the photon) in float64."""
    d = np.array([np.sin(theta), 1e-3, -side * np.cos(theta)])
    d /= np.linalg.norm(d)
    nrm = np.array([0.0, 0.0, side])
    start = np.asarray(hit) - d * (height / abs(d[2]))
    s = np.cross(d, nrm)
    s /= np.linalg.norm(s)
    p = np.cross(s, d)
    p /= np.linalg.norm(p)
    return start, d, s, p, nrm


def _fresnel(ti, n1, n2):
    """Fresnel power reflectances (R_s, R_p) for incidence angle ti, float64."""
    st = np.sin(ti) * n1 / n2
    if st >= 1.0:
        return 1.0, 1.0
    tt = np.arcsin(st)
    if ti == 0.0:
        r = ((n1 - n2) / (n1 + n2)) ** 2
        return r, r
    return (np.sin(ti - tt) / np.sin(ti + tt)) ** 2, (np.tan(ti - tt) / np.tan(ti + tt)) ** 2


FRESNEL_CASES = [   # (label, n_from, n_to, theta)
    ('near-normal', 1.0, 1.5, 0.01),
    ('20deg', 1.0, 1.5, np.radians(20.0)),
    ('45deg', 1.0, 1.5, np.radians(45.0)),
    ('brewster', 1.0, 1.5, np.arctan(1.5)),
    ('75deg', 1.0, 1.5, np.radians(75.0)),
    ('inside-20deg', 1.5, 1.0, np.radians(20.0)),
    ('inside-40deg', 1.5, 1.0, np.radians(40.0)),
    ('inside-critical+1', 1.5, 1.0, np.arcsin(1.0 / 1.5) + np.radians(1.0)),
    ('inside-60deg', 1.5, 1.0, np.radians(60.0)),
]


@pytest.mark.parametrize('backend', BACKENDS)
def test_fresnel_snell_tir(backend, request):
    n = 100000
    glass, air = _material('glass', 1.5), _material('air', 1.0)
    geo = _slab_geometry(glass, air)
    starts, dirs, pols, meta = [], [], [], []
    for label, n1, n2, theta in FRESNEL_CASES:
        side = 1.0 if n1 == 1.0 else -1.0           # outside photons come from above, inside ones from below
        start, d, s, p, nrm = _incidence(theta, n, side=side)
        for pname, pol in (('s', s), ('p', p)):
            starts.append(np.tile(start, (n, 1)))
            dirs.append(np.tile(d, (n, 1)))
            pols.append(np.tile(pol, (n, 1)))
            meta.append((label, n1, n2, pname, d, nrm))
    ph = _photons(np.concatenate(starts), np.concatenate(dirs), np.concatenate(pols))
    end = _propagate(backend, geo, ph, request=request)
    for k, (label, n1, n2, pname, d, nrm) in enumerate(meta):
        sl = slice(k * n, (k + 1) * n)
        flags = end.flags[sl]
        assert not (flags & ((1 << 15) | 1)).any(), (label, pname)          # no NaN abort, every photon hit
        refl = (flags & (1 << 6)) != 0                                        # REFLECT_SPECULAR
        d32 = d.astype(np.float32).astype(np.float64)
        ti = np.arccos(np.clip(-d32 @ nrm, -1, 1))
        rs, rp = _fresnel(ti, n1, n2)
        r = rs if pname == 's' else rp
        k_refl = int(refl.sum())
        if r >= 1.0 - 1e-12:          # total internal reflection
            assert k_refl == n, (label, pname)
        else:
            pv = scipy.stats.binomtest(k_refl, n, r).pvalue
            assert pv > P_MIN, (label, pname, k_refl / n, r, pv)
        if label == 'near-normal':    # ((n1 - n2) / (n1 + n2))^2 = 0.04 within 1e-4 of this angle's value
            assert abs(r - ((n1 - n2) / (n1 + n2)) ** 2) < 1e-4
        if label == 'brewster' and pname == 'p':
            assert k_refl == 0
        dd = end.dir[sl].astype(np.float64)
        # reflection: the mirror direction d - 2 (d.n) n (float32 rotation: 1e-5)
        mirror = d32 - 2 * (d32 @ nrm) * nrm
        if refl.any():
            assert np.abs(dd[refl] - mirror).max() < 1e-5, (label, pname)
        # refraction: Snell's law and the plane of incidence kept
        tr = ~refl
        if tr.any():
            sin_t = np.linalg.norm(np.cross(dd[tr], nrm), axis=1)
            assert np.abs(sin_t - n1 / n2 * np.sin(ti)).max() < 2e-5, (label, pname)
            assert ((dd[tr] @ nrm) < 0).all()                                  # into the other medium
            plane = np.cross(d32, nrm)
            assert np.abs(dd[tr] @ plane).max() < 2e-5
        # polarisation stays a unit vector normal to the new direction
        pp = end.pol[sl].astype(np.float64)
        assert np.abs(np.linalg.norm(pp, axis=1) - 1).max() < 1e-5
        assert np.abs((pp * dd).sum(1)).max() < 1e-5


@pytest.mark.parametrize('backend', BACKENDS)
def test_exact_normal_incidence_transmits(backend, request):
    """At exactly normal incidence the reference's sin/tan ratio is 0/0 (NaN) and
    every photon transmits (photon.h:600-605: `u < NaN` is false, the refracted
    angle is not NaN) -- the reference's own behaviour, not Fresnel's 4%."""
    n = 2000
    geo = _slab_geometry(_material('glass', 1.5), _material('air', 1.0))
    d = np.tile([0.0, 0.0, -1.0], (n, 1))
    pol = np.tile([1.0, 0.0, 0.0], (n, 1))
    # exactly axial directions are 'flat' walks (decomposed into sub-walks): keep n small
    end = _propagate(backend, geo, _photons((37.3, 21.7, 100.0), d, pol), request=request)
    assert not (end.flags & ((1 << 6) | (1 << 15))).any()
    assert np.abs(end.dir - d).max() < 1e-6         # rotated by pi - 0 about the polarisation (float pi)


def _truncated_exp_cdf(L, D):
    return lambda x: (1.0 - np.exp(-np.asarray(x) / L)) / (1.0 - np.exp(-D / L))


@pytest.mark.parametrize('backend', BACKENDS)
@pytest.mark.parametrize('process', ['absorb', 'scatter'])
def test_beer_lambert_distances(backend, process, request):
    """A photon travels an Exp(L) distance before a bulk absorption (or a
    Rayleigh scatter): fraction within the boundary D = 1 - exp(-D/L), the
    distances' KS against the truncated exponential, time = distance * n / c."""
    from chroma import make
    from chroma.geometry import Geometry, Solid
    from chroma.loader import create_geometry_from_obj
    L, nref, n = 1000.0, 1.33, 200000
    medium = _material('medium', nref, absl=L if process == 'absorb' else NOWHERE,
                       scat=L if process == 'scatter' else NOWHERE)
    g = Geometry(medium)
    g.add_solid(Solid(make.box(1e5, 1e5, 6000.0), medium, medium))          # top face at z = 3000
    geo = create_geometry_from_obj(g, update_bvh_cache=False)
    d = np.array([1e-3, 2e-3, 1.0])
    d /= np.linalg.norm(d)
    d32 = d.astype(np.float32)
    D = 3000.0 / float(d32[2])
    pol = np.cross(d, [1.0, 0.0, 0.0])
    pol /= np.linalg.norm(pol)
    end = _propagate(backend, geo, _photons((0, 0, 0), np.tile(d, (n, 1)), np.tile(pol, (n, 1))), request=request)
    bit = (1 << 1) if process == 'absorb' else (1 << 4)        # BULK_ABSORB / RAYLEIGH_SCATTER
    hit = (end.flags & bit) != 0
    pv = scipy.stats.binomtest(int(hit.sum()), n, 1.0 - np.exp(-D / L)).pvalue
    assert pv > P_MIN, (int(hit.sum()) / n, 1.0 - np.exp(-D / L))
    dist = np.linalg.norm(end.pos[hit].astype(np.float64), axis=1)
    assert scipy.stats.kstest(dist, _truncated_exp_cdf(L, D)).pvalue > P_MIN
    t = end.t[hit].astype(np.float64)
    assert np.abs(t - dist * nref / C_MM_NS).max() <= 1e-5 * t.max()
    # the others reached the boundary: at z = 3000, after D / (c / n)
    far = ~hit
    assert np.abs(end.pos[far][:, 2] - 3000.0).max() < 1e-2
    assert np.abs(end.t[far] - D * nref / C_MM_NS).max() < 1e-5 * D * nref / C_MM_NS


def _surface(name, model=0, **props):
    from chroma.geometry import Surface
    s = Surface(name, model=model)
    for k, v in props.items():
        if k in ('thickness', 'transmissive'):
            setattr(s, k, v)
        else:
            s.set(k, v)
    return s


def _random_incidence(n, seed, max_theta=np.radians(80.0)):
    """n photons onto the plane z = 0 from above at random angles < max_theta,
    random azimuths and random (unit, orthogonal) polarisations."""
    rng = np.random.default_rng(seed)
    th = np.arccos(rng.uniform(np.cos(max_theta), 1.0, n))
    ph = rng.uniform(0, 2 * np.pi, n)
    d = np.column_stack((np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), -np.cos(th)))
    hit = np.column_stack((rng.uniform(-3000, 3000, n), rng.uniform(-3000, 3000, n), np.zeros(n)))
    start = hit - d * (100.0 / np.abs(d[:, 2]))[:, None]
    r = rng.normal(size=(n, 3))
    pol = r - (r * d).sum(1)[:, None] * d
    pol /= np.linalg.norm(pol, axis=1)[:, None]
    return start, d, pol


@pytest.mark.parametrize('backend', BACKENDS)
def test_lambertian_diffuse_reflector(backend, request):
    n = 200000
    air = _material('air', 1.0)
    geo = _slab_geometry(_material('metal', 1.2), air, surface=_surface('white', reflect_diffuse=1.0))
    start, d, pol = _random_incidence(n, 5)
    end = _propagate(backend, geo, _photons(start, d, pol), request=request)
    assert ((end.flags & (1 << 5)) != 0).all()                               # REFLECT_DIFFUSE
    out = end.dir.astype(np.float64)
    c = out[:, 2]                                                            # cos to the normal facing the photon
    assert (c > 0).all()
    assert scipy.stats.kstest(c, lambda x: np.clip(x, 0, 1) ** 2).pvalue > P_MIN      # Lambert: pdf 2c
    phi = np.arctan2(out[:, 1], out[:, 0])
    assert scipy.stats.kstest(phi, scipy.stats.uniform(-np.pi, 2 * np.pi).cdf).pvalue > P_MIN
    pp = end.pol.astype(np.float64)
    assert np.abs(np.linalg.norm(pp, axis=1) - 1).max() < 1e-5 and np.abs((pp * out).sum(1)).max() < 1e-5


@pytest.mark.parametrize('backend', BACKENDS)
def test_specular_reflector_mirrors(backend, request):
    n = 100000
    geo = _slab_geometry(_material('metal', 1.2), _material('air', 1.0),
                         surface=_surface('mirror', reflect_specular=1.0))
    start, d, pol = _random_incidence(n, 6, max_theta=np.radians(89.0))
    ph = _photons(start, d, pol)
    end = _propagate(backend, geo, ph, request=request)
    assert ((end.flags & (1 << 6)) != 0).all()                               # REFLECT_SPECULAR
    d32 = ph.dir.astype(np.float64)
    mirror = d32 * np.array([1.0, 1.0, -1.0])
    assert np.abs(end.dir.astype(np.float64) - mirror).max() < 2e-5
    assert np.abs(end.pos[:, 2]).max() < 1e-3                                # reflected at the plane


def _airy(n1, n2c, n3, theta, lam, thick):
    """Single absorbing film between n1 and n3 (n2c = eta + i k, thickness
    thick): (R_s, T_s, R_p, T_p) from the Fresnel amplitudes summed over the
    film's multiple reflections (Airy), complex128, principal square roots.
    The amplitudes and the transmitted-power factor Re(n3 c3 / n1 c1) are the
    reference's conventions (photon.h:697-760: r12_p = (n2 c1 - n1 c2) /
    (n2 c1 + n1 c2), the same factor for both polarisations); the closed form
    is independent of the kernel's real-valued expansion of the sums."""
    c1 = np.cos(theta) + 0j
    s1 = np.sin(theta) + 0j
    c2 = np.sqrt(1 - (n1 / n2c) ** 2 * s1 ** 2)
    c3 = np.sqrt(1 - (n1 / n3) ** 2 * s1 ** 2 + 0j)
    beta = 2 * np.pi * thick / lam * n2c * c2                                # phase thickness of the film
    ph = np.exp(2j * beta)
    out = []
    for pol in ('s', 'p'):
        if pol == 's':
            a1, a2, a3 = n1 * c1, n2c * c2, n3 * c3
            r12, r23 = (a1 - a2) / (a1 + a2), (a2 - a3) / (a2 + a3)
            t12, t23 = 2 * a1 / (a1 + a2), 2 * a2 / (a2 + a3)
            g = (n3 * c3 / (n1 * c1)).real
        else:
            r12 = (n2c * c1 - n1 * c2) / (n2c * c1 + n1 * c2)
            r23 = (n3 * c2 - n2c * c3) / (n3 * c2 + n2c * c3)
            t12 = 2 * n1 * c1 / (n2c * c1 + n1 * c2)
            t23 = 2 * n2c * c2 / (n3 * c2 + n2c * c3)
            g = (n3 * c3 / (n1 * c1)).real
        den = 1 + r12 * r23 * ph
        r = (r12 + r23 * ph) / den
        t = t12 * t23 * np.exp(1j * beta) / den
        out += [abs(r) ** 2, g * abs(t) ** 2]
    return out


THIN_FILM_CASES = [(np.radians(0.5), 's'), (np.radians(30.0), 's'), (np.radians(30.0), 'p'),
                   (np.radians(60.0), 's'), (np.radians(60.0), 'p')]


@pytest.mark.parametrize('backend', BACKENDS)
def test_thin_film_airy(backend, request):
    """COMPLEX surface between water (n1 = 1.33, the photon's side) and glass
    (n3 = 1.5): outcome frequencies vs the Airy R / T of the film (eta 2.1,
    k 1.4, 25 nm at 400 nm): absorb = 1 - R - T, then detect with prob 0.5;
    reflect R, diffusely with prob 0.3; transmit T."""
    n, lam, thick, detect, rdiff = 200000, 400.0, 25.0, 0.5, 0.3
    film = _surface('film', model=1, detect=detect, reflect_diffuse=rdiff, eta=2.1, k=1.4, thickness=thick,
                    transmissive=1)
    geo = _slab_geometry(_material('glass', 1.5), _material('water', 1.33), surface=film)
    starts, dirs, pols, meta = [], [], [], []
    for theta, pname in THIN_FILM_CASES:
        start, d, s, p, nrm = _incidence(theta, n)
        starts.append(np.tile(start, (n, 1)))
        dirs.append(np.tile(d, (n, 1)))
        pols.append(np.tile(s if pname == 's' else p, (n, 1)))
        meta.append((theta, pname, d, nrm))
    ph = _photons(np.concatenate(starts), np.concatenate(dirs), np.concatenate(pols), wl=lam)
    end = _propagate(backend, geo, ph, request=request)
    for k, (theta, pname, d, nrm) in enumerate(meta):
        f = end.flags[k * n:(k + 1) * n]
        ti = float(np.arccos(np.clip(-d.astype(np.float32).astype(np.float64) @ nrm, -1, 1)))
        rs, ts, rp, tp = _airy(1.33, 2.1 + 1.4j, 1.5, ti, lam, thick)
        R, T = (rs, ts) if pname == 's' else (rp, tp)
        A = 1.0 - R - T
        assert 0 < A < 1 and 0 < R < 1 and 0 < T < 1
        cats = [(f & (1 << 2)) != 0, (f & (1 << 3)) != 0, (f & (1 << 5)) != 0, (f & (1 << 6)) != 0,
                (f & (1 << 8)) != 0]                      # DETECT ABSORB DIFFUSE SPECULAR TRANSMIT
        counts = np.array([c.sum() for c in cats])
        assert counts.sum() == n, (theta, pname)
        expected = np.array([A * detect, A * (1 - detect), R * rdiff, R * (1 - rdiff), T]) * n
        pv = scipy.stats.chisquare(counts, expected).pvalue
        assert pv > P_MIN, (np.degrees(theta), pname, counts / n, expected / n, pv)


@pytest.mark.parametrize('backend', BACKENDS)
def test_wls_reemission_spectrum(backend, request):
    """WLS surface absorbing and re-emitting everything: the new wavelengths
    follow the piecewise-linear reemission CDF on the wavelength grid, the new
    directions are isotropic."""
    from chroma.geometry import standard_wavelengths as wl
    n = 200000
    pdf = np.exp(-0.5 * ((wl - 480.0) / 15.0) ** 2) + 0.2 * np.exp(-0.5 * ((wl - 530.0) / 25.0) ** 2)
    cdf = np.cumsum(pdf)
    cdf = (cdf - cdf[0]) / (cdf[-1] - cdf[0])
    wls = _surface('wls', model=2, absorb=1.0, reemit=1.0, reemission_cdf=cdf)
    geo = _slab_geometry(_material('glass', 1.5), _material('air', 1.0), surface=wls)
    start, d, pol = _random_incidence(n, 8)
    end = _propagate(backend, geo, _photons(start, d, pol), request=request)
    assert ((end.flags & (1 << 7)) != 0).all()                               # SURFACE_REEMIT
    lam = end.wavelengths.astype(np.float64)
    grid = np.asarray(wl, np.float64)
    cdf32 = cdf.astype(np.float32).astype(np.float64)
    assert scipy.stats.kstest(lam, lambda x: np.interp(x, grid, cdf32)).pvalue > P_MIN
    cz = end.dir[:, 2].astype(np.float64)
    assert scipy.stats.kstest(cz, scipy.stats.uniform(-1, 2).cdf).pvalue > P_MIN
