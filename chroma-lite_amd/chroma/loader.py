"""Geometry + BVH loading (drop-in for reference chroma/loader.py:13-191).

Same geometry-string forms and cache policy as the reference, over the npz
cache of chroma.cache: BVHs are looked up by mesh MD5 (+ name) when
``read_bvh_cache``, built otherwise (``auto_build_bvh``) and saved when
``update_bvh_cache``.  The BVH is built by the host C++ builder in
libchroma_amd.so, so no GPU context is needed (the reference pushes a CUDA
context around its GPU builder, loader.py:150-152; ``cuda_device`` is accepted
and unused).
"""
import os
import sys
import time

from chroma.log import logger
from chroma.cache import Cache
from chroma.bvh import make_recursive_grid_bvh
from chroma.geometry import Geometry, Solid, Mesh, vacuum
from chroma.detector import Detector  # noqa: F401


def _cache(cache_dir):
    return Cache() if cache_dir is None else Cache(cache_dir)


def load_geometry_from_string(geometry_str, auto_build_bvh=True, read_bvh_cache=True, update_bvh_cache=True,
                              cache_dir=None, cuda_device=None):
    """'' (cached default geometry), 'name[:bvh]' (cached geometry),
    'file.stl[.bz2]', or '@module.function[:bvh]' (reference loader.py:13-129)."""
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
                                        update_bvh_cache=update_bvh_cache, cache_dir=cache_dir,
                                        cuda_device=cuda_device)
    else:
        cache = _cache(cache_dir)
        geometry = cache.load_default_geometry() if geometry_id == '' else cache.load_geometry(geometry_id)
    geometry.bvh = load_bvh(geometry, bvh_name=bvh_name, auto_build_bvh=auto_build_bvh,
                            read_bvh_cache=read_bvh_cache, update_bvh_cache=update_bvh_cache,
                            cache_dir=cache_dir, cuda_device=cuda_device)
    return geometry


def load_bvh(geometry, bvh_name='default', auto_build_bvh=True, read_bvh_cache=False, update_bvh_cache=True,
             cache_dir=None, cuda_device=None):
    """Cached BVH for the geometry's mesh MD5, or a freshly built recursive-grid
    BVH (degree 3), saved to the cache (reference loader.py:131-160)."""
    cache = _cache(cache_dir)
    mesh_hash = geometry.mesh.md5()
    bvh = None
    if read_bvh_cache and cache.exist_bvh(mesh_hash, bvh_name):
        logger.info('Loading BVH "%s" for geometry from cache.', bvh_name)
        bvh = cache.load_bvh(mesh_hash, bvh_name)
    elif auto_build_bvh:
        logger.info('Building new BVH using recursive grid algorithm.')
        t0 = time.time()
        bvh = make_recursive_grid_bvh(geometry.mesh, target_degree=3)
        logger.info('BVH generated in %1.1f seconds.', time.time() - t0)
        if update_bvh_cache:
            logger.info('Saving BVH (%s:%s) to cache.', mesh_hash, bvh_name)
            cache.save_bvh(bvh, mesh_hash, bvh_name)
    return bvh


def create_geometry_from_obj(obj, bvh_name='default', auto_build_bvh=True, read_bvh_cache=True,
                             update_bvh_cache=True, cache_dir=None, cuda_device=None):
    """Geometry / Detector / Solid / Mesh (or a callable returning one), flattened,
    with a BVH (reference loader.py:162-191)."""
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
                                read_bvh_cache=read_bvh_cache, update_bvh_cache=update_bvh_cache,
                                cache_dir=cache_dir, cuda_device=cuda_device)
    return geometry
