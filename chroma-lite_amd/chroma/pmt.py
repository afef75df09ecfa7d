"""PMT and light-collector solids from 2-D profiles (drop-in for reference
chroma/pmt.py:6-81)."""
import numpy as np

from chroma.geometry import Solid
from chroma.make import rotate_extrude
from chroma.tools import read_csv, offset


def _half_profile(profile):
    """Keep the x<0 half, mirror it to x>0, order base->face and close the
    profile on the axis."""
    profile = np.array(profile[profile[:, 0] < 0])
    profile[:, 0] = -profile[:, 0]
    profile = profile[np.argsort(profile[:, 1])]
    profile[0, 0] = 0.0
    profile[-1, 0] = 0.0
    return profile


def _load(profile_or_file):
    if isinstance(profile_or_file, str):
        return read_csv(profile_or_file)
    return np.asarray(profile_or_file, dtype=float)


def get_lc_profile(radii, a, b, d, rmin, rmax):
    c = -b * np.sqrt(1 - (rmin - d) ** 2 / a ** 2)
    return -c - b * np.sqrt(1 - (radii - d) ** 2 / a ** 2)


def build_light_collector(pmt, a, b, d, rmin, rmax, surface, npoints=10):
    if not isinstance(pmt, Solid):
        raise Exception('`pmt` must be an instance of %s' % Solid)
    radii = np.linspace(rmin, rmax, npoints)
    prof = get_lc_profile(radii, a, b, d, rmin, rmax)
    face = pmt.profile[pmt.profile[:, 1] > -1e-3]
    lc_offset = np.interp(radii[0], list(reversed(face[:, 0])), list(reversed(face[:, 1])))
    mesh = rotate_extrude(radii, prof + lc_offset, pmt.nsteps)
    return Solid(mesh, pmt.outer_material, pmt.outer_material, surface=surface)


def build_pmt_shell(filename, outer_material, glass, nsteps=16):
    profile = _half_profile(_load(filename))
    return Solid(rotate_extrude(profile[:, 0], profile[:, 1], nsteps), glass, outer_material, color=0xeeffffff)


def build_pmt(filename, glass_thickness, outer_material, glass, vacuum, photocathode_surface,
              back_surface, nsteps=16):
    """Glass envelope (profile revolved) + inner envelope (profile offset
    inwards by glass_thickness).  Inner triangles whose centre has y > 0 carry
    the photocathode surface, the rest the back surface."""
    profile = _half_profile(_load(filename))
    inner_profile = offset(profile, -glass_thickness)
    outer_mesh = rotate_extrude(profile[:, 0], profile[:, 1], nsteps)
    inner_mesh = rotate_extrude(inner_profile[:, 0], inner_profile[:, 1], nsteps)
    outer = Solid(outer_mesh, glass, outer_material)
    cathode = np.mean(inner_mesh.assemble(), axis=1)[:, 1] > 0
    surfaces = np.empty(len(cathode), dtype=object)
    surfaces[:] = [photocathode_surface if c else back_surface for c in cathode]
    inner = Solid(inner_mesh, vacuum, glass, surface=surfaces,
                  color=np.where(cathode, 0xff00, 0xff0000))
    pmt = outer + inner
    pmt.profile = profile
    pmt.outer_material = outer_material
    pmt.nsteps = nsteps
    return pmt


def build_light_collector_from_file(filename, outer_material, surface, nsteps=48):
    profile = _load(filename)
    mesh = rotate_extrude(profile[:, 0], profile[:, 1], nsteps)
    return Solid(mesh, outer_material, outer_material, surface=surface)
