"""The demo 8-inch PMT with light cone (drop-in for reference chroma/demo/pmt.py).
Profiles come from package data (data/pmt_profiles.npz: the reference's
sno_pmt.txt / sno_cone.txt point lists)."""
import os

import numpy as np

from chroma.pmt import build_pmt, build_light_collector_from_file
from chroma.demo.optics import water, glass, vacuum, shiny_surface, r7081hqe_photocathode

_PROFILES = np.load(os.path.join(os.path.dirname(__file__), 'data', 'pmt_profiles.npz'))


def build_8inch_pmt(outer_material=water, nsteps=24):
    return build_pmt(np.array(_PROFILES['sno_pmt']), 3.0, outer_material=outer_material, glass=glass,
                     vacuum=vacuum, photocathode_surface=r7081hqe_photocathode,
                     back_surface=shiny_surface, nsteps=nsteps)


def build_8inch_pmt_with_lc(outer_material=water, nsteps=24):
    pmt = build_8inch_pmt(outer_material, nsteps)
    lc = build_light_collector_from_file(np.array(_PROFILES['sno_cone']), outer_material=outer_material,
                                         surface=shiny_surface, nsteps=nsteps)
    return pmt + lc
