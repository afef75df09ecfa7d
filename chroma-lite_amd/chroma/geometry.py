"""Triangle-mesh geometry model (drop-in for reference chroma/geometry.py).

Mesh / Solid / Material / Surface / Geometry keep the reference's constructor
signatures and attributes (chroma/geometry.py:19-391).  Geometry.flatten()
produces the same flat arrays the propagator consumes: vertices, triangles,
solid_id, colors, material1_index, material2_index, surface_index
(None surface -> -1).

One intentional difference: the reference orders unique materials/surfaces by
Python set() iteration (geometry.py:114-115, id()-hash dependent, so it changes
from run to run); here the order is first appearance, which is deterministic.
Only the integer labels differ -- every triangle resolves to the same object.
"""
import hashlib

import numpy as np

from chroma.log import logger

# all material/surface properties are sampled on this grid for the device
standard_wavelengths = np.arange(60, 1000, 5).astype(np.float32)


def _first_seen(objs):
    """Unique objects in order of first appearance (identity semantics)."""
    seen, out = set(), []
    for o in objs:
        k = id(o)
        if k not in seen:
            seen.add(k)
            out.append(o)
    return out


_NATIVE_UNIQUE_MIN = 1 << 16


def _native_unique(v):
    """(unique rows, inverse) from libchroma_amd's chr_unique_vertices, or None
    when the rows hold a NaN or -0.0 (numpy then decides which duplicate stays)
    or the library cannot be loaded here (a host-only install: this host-side
    merge is the reference's np.unique either way, geometry.py:337-391)."""
    import ctypes
    try:
        from chroma.gpu import _native
        lib = _native.lib()
    except (ImportError, OSError):
        return None
    out = np.empty_like(v)
    inverse = np.empty(len(v), dtype=np.int64)
    nu = ctypes.c_uint64()
    rc = lib.chr_unique_vertices(v.ctypes.data, len(v), out.ctypes.data, ctypes.byref(nu),
                                           inverse.ctypes.data)
    if rc != 0:
        return None
    return out[:nu.value].copy(), inverse


class Mesh(object):
    """Vertices (V,3) float32 and triangles (T,3) vertex indices."""

    def __init__(self, vertices, triangles, remove_duplicate_vertices=False, round=True,
                 remove_null_triangles=True):
        vertices = np.asarray(vertices, dtype=np.float32)
        triangles = np.asarray(triangles, dtype=np.int32)
        if vertices.ndim != 2 or vertices.shape[1] != 3:
            raise ValueError('shape mismatch')
        if triangles.ndim != 2 or triangles.shape[1] != 3:
            raise ValueError('shape mismatch')
        if (triangles < 0).any():
            raise ValueError('indices in `triangles` must be positive.')
        if (triangles >= len(vertices)).any():
            raise ValueError('indices in `triangles` must be less than the length of the vertex array.')
        self.vertices = vertices
        self.triangles = triangles
        if len(vertices) == 0:
            logger.warning('Generated mesh has no vertices.')
        if len(triangles) == 0:
            logger.warning('Generated mesh has no triangles.')
        if round:
            self.vertices = self.vertices.round(decimals=12)
        if remove_duplicate_vertices:
            self.remove_duplicate_vertices()
        if remove_null_triangles:
            self.remove_null_triangles()

    def get_triangle_centers(self):
        return np.mean(self.assemble(), axis=1)

    def get_bounds(self):
        return np.min(self.vertices, axis=0), np.max(self.vertices, axis=0)

    def remove_duplicate_vertices(self):
        """Merge equal vertices, rows sorted lexicographically: np.unique over
        the (x, y, z) rows with return_inverse (reference geometry.py:71-81).
        Large meshes without NaN / -0.0 (where equal rows are bit-identical, so
        the choice of kept duplicate cannot matter) go to the parallel host sort
        chr_unique_vertices: the 170M-triangle detector's flatten spent ~45 s in
        numpy's structured argsort."""
        v = np.ascontiguousarray(self.vertices, dtype=np.float32)
        if len(v) >= _NATIVE_UNIQUE_MIN:
            got = _native_unique(v)
            if got is not None:
                self.vertices, inverse = got
                self.triangles = inverse[self.triangles]
                return
        rows = v.view([('', v.dtype)] * 3)
        uniq, inverse = np.unique(rows, return_inverse=True)
        self.vertices = uniq.view(v.dtype).reshape((len(uniq), 3))
        tri = inverse.reshape(-1)[self.triangles]
        self.triangles = tri

    def remove_null_triangles(self):
        """Drop triangles that repeat a vertex index; returns the keep-mask."""
        if len(self.triangles) == 0:
            return None
        t = self.triangles
        mask = (t[:, 0] != t[:, 1]) & (t[:, 1] != t[:, 2]) & (t[:, 0] != t[:, 2])
        self.triangles = t[mask]
        return mask

    def assemble(self, key=slice(None), group=True):
        idx = self.triangles[key] if group else self.triangles[key].flatten()
        return self.vertices[idx]

    def __add__(self, other):
        return Mesh(np.concatenate((self.vertices, other.vertices)),
                    np.concatenate((self.triangles, other.triangles + len(self.vertices))))

    def md5(self):
        h = hashlib.md5(self.vertices)
        h.update(self.triangles)
        return h.hexdigest()


def _per_triangle(value, n, dtype=object):
    if np.iterable(value) and not isinstance(value, (str, bytes)):
        if len(value) != n:
            raise ValueError('shape mismatch')
        return np.array(value, dtype=dtype)
    arr = np.empty(n, dtype=dtype)
    arr[:] = [value] * n if dtype is object else value
    return arr


class Solid(object):
    """A Mesh plus per-triangle inner material (material1), outer material
    (material2), surface and color."""

    def __init__(self, mesh, material1=None, material2=None, surface=None, color=0x33ffffff):
        self.mesh = mesh
        n = len(mesh.triangles)
        self.material1 = _per_triangle(material1, n)
        self.material2 = _per_triangle(material2, n)
        self.surface = _per_triangle(surface, n)
        self.color = _per_triangle(color, n, dtype=np.uint32)
        self.unique_materials = _first_seen(list(self.material1) + list(self.material2))
        self.unique_surfaces = _first_seen(list(self.surface))

    def __add__(self, other):
        return Solid(self.mesh + other.mesh,
                     np.concatenate((self.material1, other.material1)),
                     np.concatenate((self.material2, other.material2)),
                     np.concatenate((self.surface, other.surface)),
                     np.concatenate((self.color, other.color)))

    def _indices(self, column, lookup):
        return np.fromiter((lookup[id(o)] for o in column), dtype=np.int32, count=len(column))

    def material1_indices(self, lookup):
        return self._indices(self.material1, lookup)

    def material2_indices(self, lookup):
        return self._indices(self.material2, lookup)

    def surface_indices(self, lookup):
        return self._indices(self.surface, lookup)


class Material(object):
    """Bulk optical properties; each property is an (N,2) float32 array of
    (wavelength nm, value)."""

    def __init__(self, name='none'):
        self.name = name
        self.refractive_index = None
        self.absorption_length = None
        self.scattering_length = None
        self.scintillation_spectrum = None
        self.scintillation_light_yield = None
        self.scintillation_rise_time = None
        self.scintillation_waveform = None
        self.scintillation_mod = None
        self.comp_reemission_prob = []
        self.comp_reemission_wvl_cdf = []
        self.comp_reemission_times = []
        self.comp_reemission_time_cdf = []
        self.comp_absorption_length = []
        self.density = 0.0
        self.composition = {}

    def set(self, name, value, wavelengths=standard_wavelengths):
        if np.iterable(value):
            if len(value) != len(wavelengths):
                raise ValueError('shape mismatch')
        else:
            value = np.full(len(wavelengths), value)
        self.__dict__[name] = np.column_stack((np.asarray(wavelengths, dtype=np.float64),
                                               np.asarray(value, dtype=np.float64))).astype(np.float32)

    def __repr__(self):
        return '<Material %s>' % self.name


vacuum = Material('vacuum')
vacuum.set('refractive_index', 1.0)
vacuum.set('absorption_length', 1e6)
vacuum.set('scattering_length', 1e6)


class DichroicProps(object):
    def __init__(self, angles, reflect, transmit):
        self.angles = np.asarray(angles)
        self.dichroic_reflect = np.asarray(reflect)
        self.dichroic_transmit = np.asarray(transmit)


class AngularProps(object):
    def __init__(self, angles, transmit, reflect_specular=None, reflect_diffuse=None):
        self.angles = np.asarray(angles)
        self.transmit = np.asarray(transmit)
        self.reflect_specular = (np.asarray(reflect_specular) if reflect_specular is not None
                                 else np.zeros_like(self.transmit))
        self.reflect_diffuse = (np.asarray(reflect_diffuse) if reflect_diffuse is not None
                                else np.zeros_like(self.transmit))


class Surface(object):
    """Surface optical properties.  model: 0 default, 1 complex (thin film),
    2 WLS, 3 dichroic, 4 angular (reference geometry_types.h:22)."""

    def __init__(self, name='none', model=0):
        self.name = name
        self.model = model
        for prop in ('detect', 'absorb', 'reemit', 'reflect_diffuse', 'reflect_specular',
                     'eta', 'k', 'reemission_cdf'):
            self.set(prop, 0)
        self.dichroic_props = None
        self.angular_props = None
        self.thickness = 0.0
        self.transmissive = 0

    def set(self, name, value, wavelengths=standard_wavelengths):
        if np.iterable(value):
            if len(value) != len(wavelengths):
                raise ValueError('shape mismatch')
        else:
            value = np.full(len(wavelengths), value)
        if (np.asarray(value) < 0.0).any():
            raise Exception('all probabilities must be >= 0.0')
        self.__dict__[name] = np.column_stack((np.asarray(wavelengths, dtype=np.float64),
                                               np.asarray(value, dtype=np.float64))).astype(np.float32)

    def __repr__(self):
        return '<Surface %s>' % self.name


class Geometry(object):
    """A list of placed solids; flatten() builds the global triangle arrays."""

    def __init__(self, detector_material=None):
        self.detector_material = detector_material
        self.solids = []
        self.solid_rotations = []
        self.solid_displacements = []
        self.bvh = None

    def add_solid(self, solid, rotation=None, displacement=None):
        rotation = np.identity(3) if rotation is None else np.asarray(rotation, dtype=np.float32)
        if rotation.shape != (3, 3):
            raise ValueError('rotation matrix has the wrong shape.')
        self.solid_rotations.append(rotation.astype(np.float32))
        displacement = np.zeros(3) if displacement is None else np.asarray(displacement, dtype=np.float32)
        if displacement.shape != (3,):
            raise ValueError('displacement vector has the wrong shape.')
        self.solid_displacements.append(displacement)
        self.solids.append(solid)
        return len(self.solids) - 1

    def flatten(self):
        """Place every solid (rotate, then displace), concatenate, merge
        duplicate vertices.  Idempotent."""
        if hasattr(self, 'mesh'):
            return
        vcount = np.cumsum([0] + [len(s.mesh.vertices) for s in self.solids])
        tcount = np.cumsum([0] + [len(s.mesh.triangles) for s in self.solids])
        vertices = np.empty((vcount[-1], 3), dtype=np.float32)
        triangles = np.empty((tcount[-1], 3), dtype=np.uint32)
        logger.info('Flattening detector mesh: %d triangles, %d vertices', tcount[-1], vcount[-1])
        for i, solid in enumerate(self.solids):
            vertices[vcount[i]:vcount[i + 1]] = (np.inner(solid.mesh.vertices, self.solid_rotations[i])
                                                 + self.solid_displacements[i])
            triangles[tcount[i]:tcount[i + 1]] = solid.mesh.triangles + vcount[i]
        self.mesh = Mesh(vertices, triangles, remove_duplicate_vertices=True, remove_null_triangles=False)
        self.colors = np.concatenate([s.color for s in self.solids]) if self.solids else np.zeros(0, np.uint32)
        self.solid_id = np.concatenate([np.full(len(s.mesh.triangles), i, dtype=np.uint32)
                                        for i, s in enumerate(self.solids)]) if self.solids \
            else np.zeros(0, np.uint32)
        self.unique_materials = _first_seen([m for s in self.solids for m in s.unique_materials])
        mat_lookup = {id(m): i for i, m in enumerate(self.unique_materials)}
        # a detector places the same Solid object many times (29,007 PMTs): its
        # per-triangle index columns are computed once per distinct solid
        memo = {}

        def per_solid(s, which, lookup):
            key = (id(s), which)
            if key not in memo:
                memo[key] = getattr(s, which)(lookup)
            return memo[key]
        self.material1_index = np.concatenate([per_solid(s, 'material1_indices', mat_lookup) for s in self.solids])
        self.material2_index = np.concatenate([per_solid(s, 'material2_indices', mat_lookup) for s in self.solids])
        self.unique_surfaces = _first_seen([x for s in self.solids for x in s.unique_surfaces])
        surf_lookup = {id(x): i for i, x in enumerate(self.unique_surfaces)}
        self.surface_index = np.concatenate([per_solid(s, 'surface_indices', surf_lookup) for s in self.solids])
        none_slot = [i for i, x in enumerate(self.unique_surfaces) if x is None]
        if none_slot:
            self.surface_index[self.surface_index == none_slot[0]] = -1
