"""Scintillator detector for BASELINE config 5:
the demo PMT layout (chroma.demo.detector, reference chroma/demo/__init__.py)
filled with a two-component liquid scintillator, with the light cones cycling
through three surface models -- the demo's specular "shiny" surface
(SURFACE_DEFAULT), a dichroic filter (SURFACE_DICHROIC) and a wavelength
shifter (SURFACE_WLS) -- so every photon can take the re-emission branches of
the propagator (photon.h:500-532 bulk, 829-874 WLS, 877-907 dichroic).

The reference ships no producer for this configuration (no scintillator
material, no dichroic or WLS surface exists in its demo), so the tables below
are synthetic, physically shaped values.  As in the reference, re-emission
reuses the photon's slot: no secondary photons are spawned
(photon.h:518-532, doc/source/surface.rst:44).
"""
import numpy as np

from chroma.make import sphere
from chroma.geometry import Material, Surface, Solid, DichroicProps, standard_wavelengths
from chroma.detector import Detector
from chroma.transform import make_rotation_matrix, normalize
from chroma.pmt import build_pmt, build_light_collector_from_file
from chroma.demo import spherical_spiral
from chroma.demo.pmt import _PROFILES
from chroma.demo.optics import glass, vacuum, shiny_surface, r7081hqe_photocathode, black_surface
from chroma.log import logger

_WL = standard_wavelengths
_TIMES = np.arange(0.0, 1000.0, 0.05)


def _normalised_cdf(pdf):
    cdf = np.cumsum(pdf)
    return (cdf - cdf[0]) / (cdf[-1] - cdf[0])


def _smooth_step(x, x0, width):
    return 1.0 / (1.0 + np.exp(-(x - x0) / width))


def _exp_time_cdf(tau):
    cdf = 1.0 - np.exp(-_TIMES / tau)
    cdf[-1] = 1.0
    return np.column_stack((_TIMES, cdf))


def scintillator():
    """LAB+PPO-like liquid scintillator.  Two absorption components: the
    fluor (short absorption length below ~400 nm, re-emits with probability
    0.8 around 430 nm with a 5 ns decay) and the solvent (long absorption
    length, no re-emission).  The total absorption length is the harmonic sum
    of the components, so the bulk absorbs mostly below 400 nm and re-emits
    into the transparent region."""
    m = Material('liquid_scintillator')
    m.set('refractive_index', 1.50 + 0.01 * (450.0 / _WL) ** 2)
    fluor = 200.0 + 30000.0 * _smooth_step(_WL, 395.0, 6.0)         # mm
    solvent = 20000.0 + 60000.0 * _smooth_step(_WL, 420.0, 15.0)    # mm
    m.set('absorption_length', 1.0 / (1.0 / fluor + 1.0 / solvent))
    m.set('scattering_length', 30000.0 * (_WL / 430.0) ** 4)       # Rayleigh ~ lambda^4
    emission = _normalised_cdf(np.exp(-0.5 * ((_WL - 430.0) / 18.0) ** 2))
    flat_cdf = _normalised_cdf(np.ones(len(_WL)))
    for prob, absl, cdf, tau in ((0.8, fluor, emission, 5.0), (0.0, solvent, flat_cdf, 1.0)):
        m.comp_reemission_prob.append(np.column_stack((_WL, np.full(len(_WL), prob))).astype(np.float32))
        m.comp_reemission_wvl_cdf.append(np.column_stack((_WL, cdf)).astype(np.float32))
        m.comp_reemission_time_cdf.append(_exp_time_cdf(tau).astype(np.float32))
        m.comp_absorption_length.append(np.column_stack((_WL, absl)).astype(np.float32))
    m.density = 0.86
    m.composition = {'C': 0.8780, 'H': 0.1220}
    return m


def dichroic_surface():
    """Long-pass dichroic filter: transmits above a cut-on wavelength that
    shifts blue-ward with incidence angle, reflects below it."""
    s = Surface('dichroic_longpass', model=3)
    angles = np.linspace(0.0, np.pi / 2, 7).astype(np.float32)
    refl, trans = [], []
    for a in angles:
        cut = 450.0 - 40.0 * np.sin(a) ** 2
        t = 0.95 * _smooth_step(_WL, cut, 5.0)
        trans.append(np.column_stack((_WL, t)).astype(np.float32))
        refl.append(np.column_stack((_WL, 0.97 - t)).astype(np.float32))
    s.dichroic_props = DichroicProps(angles, refl, trans)
    return s


def wls_surface():
    """Wavelength-shifting coating: absorbs blue light and re-emits green
    (peak 490 nm); some specular/diffuse reflection, the rest transmits."""
    s = Surface('wls_coating', model=2)
    s.set('absorb', 0.6 * (1.0 - _smooth_step(_WL, 450.0, 8.0)))
    s.set('reemit', 0.85)
    s.set('reflect_specular', 0.10)
    s.set('reflect_diffuse', 0.05)
    s.set('reemission_cdf', _normalised_cdf(np.exp(-0.5 * ((_WL - 490.0) / 15.0) ** 2)))
    return s


def _pmt_with_lc(outer, lc_surface, nsteps=24):
    pmt = build_pmt(np.array(_PROFILES['sno_pmt']), 3.0, outer_material=outer, glass=glass, vacuum=vacuum,
                    photocathode_surface=r7081hqe_photocathode, back_surface=shiny_surface, nsteps=nsteps)
    lc = build_light_collector_from_file(np.array(_PROFILES['sno_cone']), outer_material=outer,
                                         surface=lc_surface, nsteps=nsteps)
    return pmt + lc


def detector(pmt_radius=14000.0, sphere_radius=14500.0, spiral_step=350.0):
    """demo.detector()'s PMT spiral (10,055 PMTs, 58.96 M triangles at the
    defaults) in liquid scintillator; light cone k uses surface k mod 3 of
    (shiny, dichroic, WLS)."""
    ls = scintillator()
    pmts = [_pmt_with_lc(ls, s) for s in (shiny_surface, dichroic_surface(), wls_surface())]
    geo = Detector(ls)
    geo.add_solid(Solid(sphere(sphere_radius, nsteps=200), ls, ls, surface=black_surface, color=0xBBFFFFFF))
    y_axis = np.array((0.0, 1.0, 0.0))
    for i, position in enumerate(spherical_spiral(pmt_radius, spiral_step)):
        direction = -normalize(position)
        rotation = make_rotation_matrix(np.arccos(np.dot(y_axis, direction)), np.cross(direction, y_axis))
        geo.add_pmt(pmts[i % 3], rotation, position)
    time_rms, charge_mean, charge_rms = 1.5, 1.0, 0.1
    geo.set_time_dist_gaussian(time_rms, -5 * time_rms, 5 * time_rms)
    geo.set_charge_dist_gaussian(charge_mean, charge_rms, 0.0, charge_mean + 5 * charge_rms)
    logger.info('Scintillator demo detector: %d PMTs', geo.num_channels())
    return geo


def tiny():
    return detector(2000.0, 2500.0, 700.0)
