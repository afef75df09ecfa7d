"""Geometry + BVH loading (drop-in for reference chroma/loader.py:13-191).

The BVH is built by the host C++ builder (no GPU needed, unlike the
reference).  Caching: BVHs are memoised in-process by mesh MD5; the on-disk
pickle cache of the reference (chroma/cache.py) is not used.
"""
import os
import sys
import time

from chroma.log import logger
from chroma.bvh import make_recursive_grid_bvh
from chroma.geometry import Geometry, Solid, Mesh, vacuum
from chroma.detector import Detector  # noqa: F401

_BVH_MEMO = {}


def load_bvh(geometry, bvh_name='default', auto_build_bvh=True, read_bvh_cache=False, update_bvh_cache=True,
             cache_dir=None, cuda_device=None):
    key = (geometry.mesh.md5(), bvh_name)
    if read_bvh_cache and key in _BVH_MEMO:
        return _BVH_MEMO[key]
    if not auto_build_bvh:
        return None
    t0 = time.time()
    bvh = make_recursive_grid_bvh(geometry.mesh, target_degree=3)
    logger.info('BVH generated in %1.1f seconds.', time.time() - t0)
    if update_bvh_cache:
        _BVH_MEMO[key] = bvh
    return bvh


def create_geometry_from_obj(obj, bvh_name='default', auto_build_bvh=True, read_bvh_cache=True,
                             update_bvh_cache=True, cache_dir=None, cuda_device=None):
    if callable(obj) and not isinstance(obj, (Geometry, Solid, Mesh)):
        obj = obj()
    if isinstance(obj, Geometry):
        geometry = obj
    elif isinstance(obj, Solid):
        geometry = Geometry()
        geometry.add_solid(obj)
    elif isinstance(obj, Mesh):
        geometry = Geometry()
        geometry.add_solid(Solid(obj, vacuum, vacuum, color=0x33ffffff))
    else:
        raise TypeError('cannot build type %s' % type(obj))
    geometry.flatten()
    if geometry.bvh is None:
        geometry.bvh = load_bvh(geometry, bvh_name=bvh_name, auto_build_bvh=auto_build_bvh,
                                read_bvh_cache=read_bvh_cache, update_bvh_cache=update_bvh_cache)
    return geometry


def load_geometry_from_string(geometry_str, auto_build_bvh=True, read_bvh_cache=True, update_bvh_cache=True,
                              cache_dir=None, cuda_device=None):
    """'@module.function[:bvh]' or 'file.stl[.bz2]'."""
    bvh_name = 'default'
    geometry_id = geometry_str
    if ':' in geometry_str:
        geometry_id, bvh_name = geometry_str.split(':')
    if os.path.exists(geometry_id) and geometry_id.lower().endswith(('.stl', '.bz2')):
        from chroma.stl import mesh_from_stl
        geometry = Geometry()
        geometry.add_solid(Solid(mesh_from_stl(geometry_id), vacuum, vacuum, color=0x33ffffff))
        geometry.flatten()
    elif geometry_id.startswith('@'):
        module_name, obj_name = geometry_id[1:].rsplit('.', 1)
        saved = list(sys.path)
        try:
            sys.path.append('.')
            module = __import__(module_name, fromlist=[obj_name])
        finally:
            sys.path = saved
        return create_geometry_from_obj(getattr(module, obj_name), bvh_name=bvh_name,
                                        auto_build_bvh=auto_build_bvh, read_bvh_cache=read_bvh_cache,
                                        update_bvh_cache=update_bvh_cache)
    else:
        raise ValueError('geometry cache lookups are not supported: %r' % geometry_str)
    geometry.bvh = load_bvh(geometry, bvh_name=bvh_name, auto_build_bvh=auto_build_bvh,
                            read_bvh_cache=read_bvh_cache, update_bvh_cache=update_bvh_cache)
    return geometry
