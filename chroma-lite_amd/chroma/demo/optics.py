"""Demo optical materials and surfaces (drop-in for reference chroma/demo/optics.py).

The numeric tables are package data (data/optics.npz), exported from the
reference by tests/golden/make_golden.py: water from WCSim, glass from the SNO+
optics database, the R7081HQE photocathode efficiency from its datasheet.
"""
import os

import numpy as np

from chroma.geometry import Material, Surface

_DATA = np.load(os.path.join(os.path.dirname(__file__), 'data', 'optics.npz'))


def _material(name):
    m = Material(name)
    for prop in ('refractive_index', 'absorption_length', 'scattering_length'):
        setattr(m, prop, np.array(_DATA['material/%s/%s' % (name, prop)]))
    return m


def _surface(name):
    s = Surface(name)
    for prop in ('detect', 'absorb', 'reemit', 'reflect_diffuse', 'reflect_specular', 'eta', 'k',
                 'reemission_cdf'):
        setattr(s, prop, np.array(_DATA['surface/%s/%s' % (name, prop)]))
    return s


vacuum = _material('vacuum')
water = _material('water')
water.density = 1.0
water.composition = {'H': 0.1119, 'O': 0.8881}
glass = _material('glass')

lambertian_surface = _surface('lambertian_surface')
black_surface = _surface('black_surface')
shiny_surface = _surface('shiny_surface')
glossy_surface = _surface('glossy_surface')
r7081hqe_photocathode = _surface('r7081hqe_photocathode')
