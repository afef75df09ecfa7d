"""Photon / channel / event containers (drop-in for reference chroma/event.py).

Field names, dtypes and constructor defaults follow the reference
(chroma/event.py:72-309) so code written against it works unchanged.
History bits are the reference's (event.py:4-16); note the device stores the
history in 16 bits, so the NAN_ABORT bit a propagated photon can carry is
NAN_ABORT_DEVICE (bit 15), see DESIGN.md.
"""
import numpy as np

NO_HIT = 1 << 0
BULK_ABSORB = 1 << 1
SURFACE_DETECT = 1 << 2
SURFACE_ABSORB = 1 << 3
RAYLEIGH_SCATTER = 1 << 4
REFLECT_DIFFUSE = 1 << 5
REFLECT_SPECULAR = 1 << 6
SURFACE_REEMIT = 1 << 7
SURFACE_TRANSMIT = 1 << 8
BULK_REEMIT = 1 << 9
CHERENKOV = 1 << 10
SCINTILLATION = 1 << 11
NAN_ABORT = 1 << 31
NAN_ABORT_DEVICE = 1 << 15


class Steps(object):
    def __init__(self, x, y, z, t, dx, dy, dz, ke, edep, qedep):
        self.x, self.y, self.z, self.t = x, y, z, t
        self.dx, self.dy, self.dz = dx, dy, dz
        self.ke, self.edep, self.qedep = ke, edep, qedep


class Vertex(object):
    """A particle vertex (name, pos, dir, kinetic energy in MeV, ...)."""

    def __init__(self, particle_name, pos, dir, ke, t0=0.0, pol=None, steps=None,
                 children=None, trackid=-1, pdgcode=-1):
        self.particle_name = particle_name
        self.pos, self.dir, self.pol = pos, dir, pol
        self.ke, self.t0 = ke, t0
        self.steps, self.children = steps, children
        self.trackid, self.pdgcode = trackid, pdgcode

    def __str__(self):
        return 'Vertex(%s,ke=%s,steps=%s)' % (self.particle_name, self.ke, bool(self.steps))

    __repr__ = __str__


_FIELDS = ('pos', 'dir', 'pol', 'wavelengths', 't', 'last_hit_triangles', 'flags',
           'weights', 'evidx', 'channel')


class Photons(object):
    """A list of n photons stored as parallel numpy arrays.

    pos, dir, pol: float32 (n,3); wavelengths (nm), t (ns): float32 (n,);
    last_hit_triangles: int32 (default -1); flags: uint32 (default 0);
    weights: float32 (default 1); evidx: uint32 (default 0); channel: uint32.
    """

    def __init__(self, pos=np.empty((0, 3)), dir=np.empty((0, 3)), pol=np.empty((0, 3)),
                 wavelengths=np.empty((0)), t=None, last_hit_triangles=None, flags=None,
                 weights=None, evidx=None, channel=None):
        self.pos = np.asarray(pos, dtype=np.float32)
        self.dir = np.asarray(dir, dtype=np.float32)
        self.pol = np.asarray(pol, dtype=np.float32)
        self.wavelengths = np.asarray(wavelengths, dtype=np.float32)
        n = len(pos)

        def field(value, dtype, default):
            if value is None:
                return np.full(n, default, dtype=dtype)
            return np.asarray(value, dtype=dtype)

        self.t = field(t, np.float32, 0)
        self.last_hit_triangles = field(last_hit_triangles, np.int32, -1)
        self.flags = field(flags, np.uint32, 0)
        self.weights = field(weights, np.float32, 1)
        self.evidx = field(evidx, np.uint32, 0)
        self.channel = field(channel, np.uint32, 0)

    @staticmethod
    def join(photon_list, concatenate=True):
        """Concatenate many Photons (or stack per-step scalars if concatenate=False)."""
        combine = np.concatenate if concatenate else np.asarray
        arrays = [combine([getattr(p, f) for p in photon_list]) for f in _FIELDS]
        return Photons(*arrays)

    def __add__(self, other):
        return Photons(*[np.concatenate((getattr(self, f), getattr(other, f))) for f in _FIELDS])

    def __len__(self):
        return len(self.pos)

    def __str__(self):
        if len(self.pos) == 1:
            return ('Photon(pos=%s,dir=%s,pol=%s,wavelength=%s,t=%s,last_hit_triangle=%s,'
                    'flag=%s,weight=%s)' % (self.pos[0], self.dir[0], self.pol[0],
                                            self.wavelengths[0], self.t[0],
                                            self.last_hit_triangles[0], self.flags[0],
                                            self.weights[0]))
        return 'Photons[%d]' % len(self.pos)

    __repr__ = __str__

    def __getitem__(self, key):
        return Photons(*[getattr(self, f)[key] for f in _FIELDS])

    def reduced(self, reduction_factor=1.0):
        n = len(self)
        choice = np.random.permutation(n)[:int(n * reduction_factor)]
        return self[choice]


class Channels(object):
    """Per-channel readout: hit (bool), t (ns), q, flags (OR of photon histories)."""

    def __init__(self, hit, t, q, flags=None, evidx=None):
        self.hit, self.t, self.q, self.flags, self.evidx = hit, t, q, flags, evidx

    def hit_channels(self, return_flags=False):
        ids = self.hit.nonzero()[0]
        if return_flags:
            return ids, self.t[self.hit], self.q[self.hit], self.flags[self.hit]
        return ids, self.t[self.hit], self.q[self.hit]


class Event(object):
    def __init__(self, id=0, vertices=None, photons_beg=None, photons_end=None,
                 photon_tracks=None, photon_parent_trackids=None, hits=None,
                 flat_hits=None, channels=None):
        self.id = id
        self.nphotons = None
        if vertices is None:
            self.vertices = []
        elif np.iterable(vertices):
            self.vertices = vertices
        else:
            self.vertices = [vertices]
        self.photons_beg = photons_beg
        self.photons_end = photons_end
        self.photon_tracks = photon_tracks
        self.photon_parent_trackids = photon_parent_trackids
        self.hits = hits
        self.flat_hits = flat_hits
        self.channels = channels
