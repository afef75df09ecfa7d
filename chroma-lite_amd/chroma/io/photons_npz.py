"""Photon archives of ``chroma-profile --photons-npz`` (reference
bin/chroma-profile:226-251).

Required arrays: pos (N,3), dir (N,3), pol (N,3), wavelengths (N,).
Optional: t (zeros when missing), last_hit_triangles, flags, weights, evidx
(event.Photons defaults when missing).  Loaded with allow_pickle=False.

Difference: the reference's ``pick(name, default=None)`` raises KeyError for
a missing optional array (its ``default is not None`` test never passes for
None), so an archive without, e.g., ``flags`` fails there; here the optional
arrays are optional, as the reference's own call intends.
"""
import numpy as np

from chroma import event

REQUIRED = ('pos', 'dir', 'pol', 'wavelengths')
OPTIONAL = ('last_hit_triangles', 'flags', 'weights', 'evidx')


def load_photons_npz(path):
    with np.load(path, allow_pickle=False) as data:
        missing = sorted(set(REQUIRED) - set(data.files))
        if missing:
            raise RuntimeError('%s is missing required arrays: %s' % (path, ', '.join(missing)))
        kw = {k: data[k] for k in REQUIRED}
        kw['t'] = data['t'] if 't' in data.files else np.zeros(len(data['pos']), dtype=np.float32)
        for k in OPTIONAL:
            kw[k] = data[k] if k in data.files else None
    return event.Photons(**kw)


def save_photons_npz(path, photons):
    """Write every Photons field (the loader reads them back unchanged)."""
    np.savez(path, pos=photons.pos, dir=photons.dir, pol=photons.pol, wavelengths=photons.wavelengths,
             t=photons.t, last_hit_triangles=photons.last_hit_triangles, flags=photons.flags,
             weights=photons.weights, evidx=photons.evidx)


def synthetic_photons(nphotons, seed=None):
    """chroma-profile's synthetic source (reference bin/chroma-profile:206-223):
    positions uniform in a 2 m cube around the origin, isotropic directions,
    polarisations perpendicular to them, wavelengths U[380, 500) nm, t = 0."""
    rng = np.random.default_rng(seed)
    pos = rng.uniform(-1000.0, 1000.0, size=(nphotons, 3)).astype(np.float32)
    directions = rng.normal(size=(nphotons, 3))
    directions /= np.linalg.norm(directions, axis=1)[:, None]
    directions = directions.astype(np.float32)
    random_vec = rng.normal(size=(nphotons, 3))
    pol = random_vec - (random_vec * directions).sum(axis=1)[:, None] * directions
    pol /= np.linalg.norm(pol, axis=1)[:, None]
    pol = pol.astype(np.float32)
    wavelengths = rng.uniform(380.0, 500.0, size=nphotons).astype(np.float32)
    t = np.zeros(nphotons, dtype=np.float32)
    return event.Photons(pos, directions, pol, wavelengths, t)
