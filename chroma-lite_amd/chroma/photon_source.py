"""Synthetic photon sources for tests and benchmarks.

isotropic() is the BASELINE.md measurement input: a point source with
dir = normalised N(0,1)^3, pol = a random vector made orthogonal to dir and
normalised, wavelength ~ U[380, 500) nm, t = 0, flags = 0, last_hit = -1,
weight = 1, evidx = 0, drawn from numpy.random.default_rng(seed).
"""
import numpy as np

from chroma.event import Photons


def isotropic(n, seed=20260102, pos=(0.0, 0.0, 0.0), wavelength_range=(380.0, 500.0)):
    rng = np.random.default_rng(seed)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    r = rng.normal(size=(n, 3))
    p = r - (r * d).sum(axis=1)[:, None] * d
    p /= np.linalg.norm(p, axis=1)[:, None]
    wl = rng.uniform(wavelength_range[0], wavelength_range[1], size=n)
    position = np.tile(np.asarray(pos, dtype=np.float32), (n, 1))
    return Photons(position, d.astype(np.float32), p.astype(np.float32), wl.astype(np.float32))
