"""On-disk geometry and BVH cache (drop-in for reference chroma/cache.py:1-246).

Same directory layout and API as the reference -- ``<cache_dir>/geo/<name>``
for flattened geometries, ``<cache_dir>/bvh/<mesh md5>/<name>`` for BVHs,
``geo/.default`` a symlink to the default geometry, ``$CHROMA_CACHE_DIR`` or
``~/.chroma`` -- but the files are numpy ``.npz`` archives loaded with
``allow_pickle=False`` instead of pickles (cache.py:12,112-116,219-236), so
reading a cache executes nothing from it.  A geometry file holds the flattened
arrays the propagator consumes (vertices, triangles, solid_id, colors,
material/surface indices), every unique material and surface property table,
the detector channel maps and time/charge CDFs, and the mesh MD5 (read alone
by get_geometry_hash, as cache.py:141-151).  As in the reference, the BVH and
the placed solids are not saved with a geometry (cache.py:105-110).  The
traversal BVH the kernels walk is cached beside the reference BVH it was
built from (``bvh/<md5>/<name>.wide/``, chroma.gpu.wide_bvh); a BVH loaded or
saved here carries ``cache_ref`` to find it.
"""
import json
import os

import numpy as np

from chroma.log import logger

cache_dir = os.environ.get('CHROMA_CACHE_DIR', os.path.expanduser('~/.chroma/'))

FORMAT = 'chroma-lite_amd.cache.v1'


class GeometryNotFoundError(Exception):
    """A requested geometry was not found in the on-disk cache."""

    def __init__(self, msg):
        Exception.__init__(self, msg)


class BVHNotFoundError(Exception):
    """A requested bounding volume hierarchy was not found in the on-disk cache."""

    def __init__(self, msg):
        Exception.__init__(self, msg)


def verify_or_create_dir(dirname, exception_msg, logger_msg=None):
    """Create ``dirname`` if missing; IOError if it exists and is not a directory
    (reference cache.py:30-44)."""
    if not os.path.isdir(dirname):
        if os.path.exists(dirname):
            raise IOError(exception_msg)
        if logger_msg is not None:
            logger.info(logger_msg)
        try:
            os.mkdir(dirname)
        except FileExistsError:     # another process (one per GPU) made it first
            if not os.path.isdir(dirname):
                raise IOError(exception_msg)


# ------------------------------------------------------------ (de)serialisation
_MATERIAL_TABLES = ('refractive_index', 'absorption_length', 'scattering_length', 'scintillation_spectrum',
                    'scintillation_light_yield', 'scintillation_rise_time', 'scintillation_waveform',
                    'scintillation_mod')
_MATERIAL_LISTS = ('comp_reemission_prob', 'comp_reemission_wvl_cdf', 'comp_reemission_times',
                   'comp_reemission_time_cdf', 'comp_absorption_length')
_SURFACE_TABLES = ('detect', 'absorb', 'reemit', 'reflect_diffuse', 'reflect_specular', 'eta', 'k',
                   'reemission_cdf')


def _put(arrays, key, value):
    if value is None:
        return None
    a = np.asarray(value)
    if a.dtype == object:
        raise TypeError('cannot cache object array %s' % key)
    arrays[key] = a
    return key


def _encode_material(m, i, arrays):
    if m is None:
        return None
    d = {'name': m.name, 'density': float(getattr(m, 'density', 0.0)),
         'composition': {str(k): float(v) for k, v in getattr(m, 'composition', {}).items()},
         'tables': {}, 'lists': {}}
    for p in _MATERIAL_TABLES:
        k = _put(arrays, 'm%s.%s' % (i, p), getattr(m, p, None))
        if k:
            d['tables'][p] = k
    for p in _MATERIAL_LISTS:
        d['lists'][p] = [_put(arrays, 'm%s.%s.%d' % (i, p, j), v) for j, v in enumerate(getattr(m, p, []) or [])]
    return d


def _decode_material(d, z):
    from chroma.geometry import Material
    if d is None:
        return None
    m = Material(d['name'])
    m.density = d['density']
    m.composition = dict(d['composition'])
    for p, k in d['tables'].items():
        setattr(m, p, z[k])
    for p, keys in d['lists'].items():
        setattr(m, p, [z[k] for k in keys])
    return m


def _encode_surface(s, i, arrays):
    if s is None:
        return None
    d = {'name': s.name, 'model': int(s.model), 'thickness': float(s.thickness),
         'transmissive': int(s.transmissive), 'tables': {}, 'dichroic': None, 'angular': None}
    for p in _SURFACE_TABLES:
        k = _put(arrays, 's%s.%s' % (i, p), getattr(s, p, None))
        if k:
            d['tables'][p] = k
    dp = getattr(s, 'dichroic_props', None)
    if dp is not None:
        d['dichroic'] = {'angles': _put(arrays, 's%s.dichroic.angles' % i, dp.angles),
                         'reflect': _put(arrays, 's%s.dichroic.reflect' % i, np.asarray(dp.dichroic_reflect)),
                         'transmit': _put(arrays, 's%s.dichroic.transmit' % i, np.asarray(dp.dichroic_transmit))}
    ap = getattr(s, 'angular_props', None)
    if ap is not None:
        d['angular'] = {p: _put(arrays, 's%s.angular.%s' % (i, p), getattr(ap, p))
                        for p in ('angles', 'transmit', 'reflect_specular', 'reflect_diffuse')}
    return d


def _decode_surface(d, z):
    from chroma.geometry import Surface, DichroicProps, AngularProps
    if d is None:
        return None
    s = Surface(d['name'], model=d['model'])
    s.thickness = d['thickness']
    s.transmissive = d['transmissive']
    for p, k in d['tables'].items():
        setattr(s, p, z[k])
    if d['dichroic']:
        c = d['dichroic']
        s.dichroic_props = DichroicProps(z[c['angles']], z[c['reflect']], z[c['transmit']])
    if d['angular']:
        c = d['angular']
        s.angular_props = AngularProps(z[c['angles']], z[c['transmit']], z[c['reflect_specular']],
                                       z[c['reflect_diffuse']])
    return s


_WIRE_OBJECTS = {'surface': 'surfaces', 'material_inner': 'materials', 'material_outer': 'materials'}


def _encode_wireplane(p, i, mats, surfs, arrays):
    """Analytic wire plane (dict of numbers + surface/material objects, the
    reference's WirePlane, geometry_types.h:42-58): numbers as JSON, objects
    as an index into the geometry's unique lists or inlined."""
    d = {}
    for k, v in p.items():
        if k in _WIRE_OBJECTS:
            pool = surfs if _WIRE_OBJECTS[k] == 'surfaces' else mats
            idx = [j for j, o in enumerate(pool) if o is v]
            if v is None:
                d[k] = None
            elif idx:
                d[k] = {'index': idx[0]}
            elif _WIRE_OBJECTS[k] == 'surfaces':
                d[k] = {'inline': _encode_surface(v, 'w%d%s' % (i, k), arrays)}
            else:
                d[k] = {'inline': _encode_material(v, 'w%d%s' % (i, k), arrays)}
        else:
            d[k] = np.asarray(v, dtype=np.float64).tolist()
    return d


def _decode_wireplane(d, mats, surfs, z):
    p = {}
    for k, v in d.items():
        if k in _WIRE_OBJECTS:
            if v is None:
                p[k] = None
            elif 'index' in v:
                p[k] = (surfs if _WIRE_OBJECTS[k] == 'surfaces' else mats)[v['index']]
            else:
                p[k] = (_decode_surface if _WIRE_OBJECTS[k] == 'surfaces' else _decode_material)(v['inline'], z)
        else:
            p[k] = tuple(v) if isinstance(v, list) else v
    return p


_FLAT = ('solid_id', 'colors', 'material1_index', 'material2_index', 'surface_index')
_DETECTOR = ('solid_id_to_channel_index', 'channel_index_to_solid_id', 'channel_index_to_channel_type',
             'channel_index_to_position')


def geometry_to_arrays(geometry):
    """Flattened geometry -> (dict of arrays, JSON-able manifest)."""
    from chroma.detector import Detector
    geometry.flatten()
    arrays = {'vertices': geometry.mesh.vertices, 'triangles': geometry.mesh.triangles}
    for k in _FLAT:
        arrays[k] = np.asarray(getattr(geometry, k))
    mats = list(geometry.unique_materials)
    man = {'format': FORMAT, 'md5': geometry.mesh.md5(), 'detector': isinstance(geometry, Detector),
           'materials': [_encode_material(m, i, arrays) for i, m in enumerate(mats)],
           'surfaces': [_encode_surface(s, i, arrays) for i, s in enumerate(geometry.unique_surfaces)],
           'detector_material': None}
    dm = geometry.detector_material
    if dm is not None:
        idx = [i for i, m in enumerate(mats) if m is dm]
        if idx:
            man['detector_material'] = {'index': idx[0]}
        else:
            man['detector_material'] = {'inline': _encode_material(dm, len(mats), arrays)}
    man['wireplanes'] = [_encode_wireplane(p, i, mats, list(geometry.unique_surfaces), arrays)
                         for i, p in enumerate(getattr(geometry, 'wireplanes', None) or [])]
    if man['detector']:
        for k in _DETECTOR:
            arrays[k] = np.asarray(getattr(geometry, k))
        arrays['time_cdf.x'], arrays['time_cdf.y'] = (np.asarray(a) for a in geometry.time_cdf)
        arrays['charge_cdf.x'], arrays['charge_cdf.y'] = (np.asarray(a) for a in geometry.charge_cdf)
    return arrays, man


def geometry_from_arrays(z, man):
    from chroma.geometry import Geometry, Mesh
    from chroma.detector import Detector
    if man.get('format') != FORMAT:
        raise IOError('unknown geometry cache format %r' % man.get('format'))
    mats = [_decode_material(d, z) for d in man['materials']]
    geo = Detector() if man['detector'] else Geometry()
    dm = man['detector_material']
    if dm is not None:
        geo.detector_material = mats[dm['index']] if 'index' in dm else _decode_material(dm['inline'], z)
    mesh = Mesh.__new__(Mesh)
    mesh.vertices, mesh.triangles = z['vertices'], z['triangles']
    geo.mesh = mesh
    for k in _FLAT:
        setattr(geo, k, z[k])
    geo.unique_materials = mats
    geo.unique_surfaces = [_decode_surface(d, z) for d in man['surfaces']]
    if man.get('wireplanes'):
        geo.wireplanes = [_decode_wireplane(d, mats, geo.unique_surfaces, z) for d in man['wireplanes']]
    if man['detector']:
        for k in _DETECTOR:
            setattr(geo, k, z[k])
        geo.time_cdf = (z['time_cdf.x'], z['time_cdf.y'])
        geo.charge_cdf = (z['charge_cdf.x'], z['charge_cdf.y'])
    return geo


def _write_npz(path, arrays):
    # unique temporary name: concurrent writers (one process per GPU) never share it
    tmp = '%s.%d.tmp.npz' % (path, os.getpid())
    np.savez(tmp, **arrays)
    os.replace(tmp, path)


class Cache(object):
    """A Chroma cache directory (reference cache.py:46-246).  Geometry names and
    BVH names map directly to file names."""

    def __init__(self, cache_dir=cache_dir):
        self.cache_dir = cache_dir
        verify_or_create_dir(self.cache_dir,
                             exception_msg='Path for cache already exists, but is not a directory: %s' % cache_dir,
                             logger_msg='Creating new Chroma cache directory at %s' % cache_dir)
        self.geo_dir = os.path.join(cache_dir, 'geo')
        verify_or_create_dir(self.geo_dir, exception_msg='Path for geometry directory in cache already exists, '
                                                         'but is not a directory: %s' % self.geo_dir)
        self.bvh_dir = os.path.join(cache_dir, 'bvh')
        verify_or_create_dir(self.bvh_dir, exception_msg='Path for BVH directory in cache already exists, '
                                                         'but is not a directory: %s' % self.bvh_dir)

    # -- geometry
    def get_geometry_filename(self, name):
        return os.path.join(self.geo_dir, name)

    def list_geometry(self):
        return [n for n in os.listdir(self.geo_dir) if not n.endswith('.tmp.npz')]

    def save_geometry(self, name, geometry):
        arrays, man = geometry_to_arrays(geometry)
        arrays['__manifest__'] = np.array(json.dumps(man))
        arrays['__md5__'] = np.array(man['md5'])
        _write_npz(self.get_geometry_filename(name), arrays)

    def load_geometry(self, name):
        geo_file = self.get_geometry_filename(name)
        if not os.path.exists(geo_file):
            raise GeometryNotFoundError(name)
        with np.load(geo_file, allow_pickle=False) as f:
            z = {k: f[k] for k in f.files}
        return geometry_from_arrays(z, json.loads(str(z['__manifest__'])))

    def remove_geometry(self, name):
        geo_file = self.get_geometry_filename(name)
        if os.path.exists(geo_file):
            os.remove(geo_file)

    def get_geometry_hash(self, name):
        geo_file = self.get_geometry_filename(name)
        if not os.path.exists(geo_file):
            raise GeometryNotFoundError(name)
        with np.load(geo_file, allow_pickle=False) as f:
            return str(f['__md5__'])

    def load_default_geometry(self):
        return self.load_geometry('.default')

    def set_default_geometry(self, name):
        default_geo_file = self.get_geometry_filename('.default')
        geo_file = self.get_geometry_filename(name)
        if not os.path.exists(geo_file):
            raise GeometryNotFoundError(name)
        if os.path.lexists(default_geo_file):
            if os.path.islink(default_geo_file):
                os.remove(default_geo_file)
            else:
                raise IOError('Non-symlink found where expected a symlink: ' + default_geo_file)
        os.symlink(geo_file, default_geo_file)

    # -- BVH
    def get_bvh_directory(self, mesh_hash):
        return os.path.join(self.bvh_dir, mesh_hash)

    def get_bvh_filename(self, mesh_hash, name='default'):
        return os.path.join(self.get_bvh_directory(mesh_hash), name)

    def list_bvh(self, mesh_hash):
        bvh_dir = self.get_bvh_directory(mesh_hash)
        if not os.path.isdir(bvh_dir):
            return []
        # BVH files only: the traversal BVHs cached beside them are directories
        # (<name>.wide/, chroma.gpu.wide_bvh)
        return [n for n in os.listdir(bvh_dir)
                if not n.endswith('.tmp.npz') and os.path.isfile(os.path.join(bvh_dir, n))]

    def exist_bvh(self, mesh_hash, name='default'):
        return os.path.isfile(self.get_bvh_filename(mesh_hash, name))

    def save_bvh(self, bvh, mesh_hash, name='default'):
        bvh_dir = self.get_bvh_directory(mesh_hash)
        verify_or_create_dir(bvh_dir, exception_msg='Non-directory already exists where BVH directory should go: '
                                                    + bvh_dir)
        # the traversal BVHs derived from the BVH this one replaces go with it (their
        # fingerprint would refuse them anyway)
        wide_dir = self.get_bvh_filename(mesh_hash, name) + '.wide'
        if os.path.isdir(wide_dir):
            import shutil
            shutil.rmtree(wide_dir, ignore_errors=True)
        _write_npz(self.get_bvh_filename(mesh_hash, name),
                   {'nodes': bvh.nodes, 'layer_offsets': np.asarray(bvh.layer_offsets, dtype=np.int64),
                    'world_origin': np.asarray(bvh.world_coords.world_origin),
                    'world_scale': np.asarray(bvh.world_coords.world_scale)})
        bvh.cache_ref = (self.cache_dir, mesh_hash, name)

    def load_bvh(self, mesh_hash, name='default'):
        from chroma.bvh import BVH, WorldCoords
        bvh_file = self.get_bvh_filename(mesh_hash, name)
        if not os.path.exists(bvh_file):
            raise BVHNotFoundError(mesh_hash + ':' + name)
        with np.load(bvh_file, allow_pickle=False) as z:
            bvh = BVH(WorldCoords(z['world_origin'], z['world_scale'][()]), z['nodes'],
                      [int(x) for x in z['layer_offsets']])
        # where the traversal BVH derived from this one is cached (chroma.gpu.wide_bvh)
        bvh.cache_ref = (self.cache_dir, mesh_hash, name)
        return bvh

    def remove_bvh(self, mesh_hash, name='default'):
        bvh_file = self.get_bvh_filename(mesh_hash, name)
        if os.path.exists(bvh_file):
            os.remove(bvh_file)
        wide_dir = bvh_file + '.wide'      # the traversal BVHs derived from it
        if os.path.isdir(wide_dir):
            import shutil
            shutil.rmtree(wide_dir, ignore_errors=True)
