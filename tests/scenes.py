"""Synthetic scenes that exercise every branch of the photon physics:
bulk absorption + Rayleigh scattering + multi-component bulk re-emission
(photon.h:455-570), Fresnel (572-632), the default surface model (953-1037),
thin-film COMPLEX (669-827), WLS (829-874), DICHROIC (877-907),
ANGULAR (909-951) and analytic FP64 wire planes (108-270)."""
import numpy as np

from chroma import make
from chroma.detector import Detector
from chroma.geometry import Material, Surface, Solid, DichroicProps, AngularProps, standard_wavelengths


def _material(name, n, absl, scat):
    m = Material(name)
    m.set('refractive_index', n)
    m.set('absorption_length', absl)
    m.set('scattering_length', scat)
    return m


def materials():
    water = _material('water', 1.33, 3000.0, 2000.0)
    glass = _material('glass', 1.5, 1000.0, 1e6)
    metal = _material('metal', 1.2, 1.0, 1e6)
    scint = _material('scint', 1.45, 800.0, 1500.0)
    wl = standard_wavelengths
    # two components; reemission spectrum peaked near 430 nm
    pdf = np.exp(-0.5 * ((wl - 430.0) / 20.0) ** 2)
    cdf = np.cumsum(pdf)
    cdf = (cdf - cdf[0]) / (cdf[-1] - cdf[0])
    times = np.arange(0, 1000, 0.05)
    tcdf = 1.0 - np.exp(-times / 5.0)
    tcdf[-1] = 1.0
    for prob, absl in ((0.8, 1200.0), (0.3, 2400.0)):
        scint.comp_reemission_prob.append(np.column_stack((wl, np.full(len(wl), prob))))
        scint.comp_reemission_wvl_cdf.append(np.column_stack((wl, cdf)))
        scint.comp_reemission_time_cdf.append(np.column_stack((times, tcdf)))
        scint.comp_absorption_length.append(np.column_stack((wl, np.full(len(wl), absl))))
    return dict(water=water, glass=glass, metal=metal, scint=scint)


def surfaces():
    wl = standard_wavelengths
    black = Surface('black')
    black.set('absorb', 1.0)
    pmt = Surface('cathode')
    pmt.set('detect', 0.4)
    pmt.set('absorb', 0.3)
    pmt.set('reflect_diffuse', 0.2)
    pmt.set('reflect_specular', 0.05)          # 5% PASS
    film = Surface('film', model=1)
    film.set('detect', 0.5)
    film.set('reflect_diffuse', 0.3)
    film.set('eta', 2.1)
    film.set('k', 1.4)
    film.thickness = 25.0
    film.transmissive = 1
    wls = Surface('wls', model=2)
    wls.set('absorb', 0.5)
    wls.set('reemit', 0.7)
    wls.set('reflect_specular', 0.1)
    wls.set('reflect_diffuse', 0.1)
    pdf = np.exp(-0.5 * ((wl - 480.0) / 15.0) ** 2)
    cdf = np.cumsum(pdf)
    wls.set('reemission_cdf', (cdf - cdf[0]) / (cdf[-1] - cdf[0]))
    dich = Surface('dichroic', model=3)
    angles = np.array([0.0, 0.5, 1.0, 1.5707964])
    refl = [np.column_stack((wl, np.clip((wl - 300.0) / 400.0 * (1 + a) / 3.0, 0, 1))) for a in angles]
    trans = [np.column_stack((wl, np.clip(0.9 - r[:, 1], 0, 1))) for r in refl]
    dich.dichroic_props = DichroicProps(angles, refl, trans)
    ang = Surface('angular', model=4)
    ang.angular_props = AngularProps(np.array([0.0, 0.4, 0.8, 1.2, 1.5707964]),
                                     np.array([0.6, 0.5, 0.4, 0.2, 0.0]),
                                     np.array([0.1, 0.2, 0.2, 0.3, 0.5]),
                                     np.array([0.1, 0.1, 0.2, 0.2, 0.3]))
    mirror = Surface('mirror')
    mirror.set('reflect_specular', 0.97)
    mirror.set('absorb', 0.03)
    return dict(black=black, pmt=pmt, film=film, wls=wls, dich=dich, ang=ang, mirror=mirror)


def physics_scene(wireplanes=True):
    m = materials()
    s = surfaces()
    det = Detector(m['water'])
    # outer black box (inside: water)
    det.add_solid(Solid(make.box(4000.0, 4000.0, 4000.0), m['water'], m['water'], surface=s['black']))
    # scintillator slab with plain Fresnel boundary
    det.add_solid(Solid(make.box(1200.0, 1200.0, 300.0), m['scint'], m['water']), displacement=(0, 0, -900))
    # glass sphere with thin-film surface, a PMT channel
    det.add_pmt(Solid(make.sphere(300.0, nsteps=24), m['glass'], m['water'], surface=s['film']),
                displacement=(900, 0, 0))
    # WLS plate, dichroic plate, angular plate, mirror plate, cathode cube
    det.add_solid(Solid(make.box(600.0, 600.0, 60.0), m['glass'], m['water'], surface=s['wls']),
                  displacement=(-900, 0, 300))
    det.add_solid(Solid(make.box(60.0, 700.0, 700.0), m['glass'], m['water'], surface=s['dich']),
                  displacement=(0, 900, 0))
    det.add_solid(Solid(make.box(700.0, 60.0, 700.0), m['glass'], m['water'], surface=s['ang']),
                  displacement=(0, -900, 200))
    det.add_solid(Solid(make.box(800.0, 800.0, 40.0), m['metal'], m['water'], surface=s['mirror']),
                  displacement=(0, 0, 1500))
    det.add_pmt(Solid(make.box(300.0, 300.0, 300.0), m['glass'], m['water'], surface=s['pmt']),
                displacement=(-900, -900, -300))
    det.add_pmt(Solid(make.cube(200.0), m['glass'], m['water']), displacement=(900, 900, 900))
    det.set_time_dist_gaussian(1.2, -6.0, 6.0)
    det.set_charge_dist_gaussian(1.0, 0.1, 0.0, 1.5)
    if wireplanes:
        det.wireplanes = [dict(origin=(0.0, 0.0, 600.0), u=(1.0, 0.0, 0.0), v=(0.0, 1.0, 0.0), pitch=40.0,
                               radius=3.0, umin=-700.0, umax=700.0, vmin=-700.0, vmax=700.0, v0=0.0,
                               surface=s['mirror'], material_inner=m['metal'], material_outer=m['water'])]
    return det


def photon_sources(n, seed=7):
    """Isotropic photons from several points inside the scene."""
    from chroma.photon_source import isotropic
    from chroma.event import Photons
    centres = [(0, 0, 0), (500, 300, -200), (-300, -500, 800), (200, -200, -700)]
    parts = [isotropic(n // len(centres) + (1 if i < n % len(centres) else 0), seed=seed + i, pos=c,
                       wavelength_range=(300.0, 600.0)) for i, c in enumerate(centres)]
    return Photons.join(parts)


def camera_rays(width, height, position, look_at, fov_deg=40.0, up=(0.0, 0.0, 1.0)):
    """Pinhole-camera rays (camera.py-style): one per pixel, unit directions,
    float32 (positions all `position`)."""
    position = np.asarray(position, np.float64)
    forward = np.asarray(look_at, np.float64) - position
    forward /= np.linalg.norm(forward)
    right = np.cross(forward, np.asarray(up, np.float64))
    right /= np.linalg.norm(right)
    upv = np.cross(right, forward)
    half = np.tan(np.radians(fov_deg) / 2)
    xs = (np.arange(width) + 0.5) / width * 2 - 1
    ys = (np.arange(height) + 0.5) / height * 2 - 1
    gx, gy = np.meshgrid(xs * half * width / height, ys * half)
    d = forward[None, :] + gx.reshape(-1, 1) * right[None, :] + gy.reshape(-1, 1) * upv[None, :]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pos = np.tile(position, (len(d), 1))
    return pos.astype(np.float32), d.astype(np.float32)
