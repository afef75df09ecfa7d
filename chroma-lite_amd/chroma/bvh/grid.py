"""Recursive-grid BVH builder (reference chroma/bvh/grid.py:11-95), executed by
the host C++ builder chr_bvh_build_grid (chroma-lite_amd/csrc/bvh_build.cpp)."""
import ctypes

import numpy as np

from chroma.bvh.bvh import BVH, WorldCoords, uint4


def make_recursive_grid_bvh(mesh, target_degree=3, verbose=False):
    """Leaves (one per triangle, quantised, Morton ordered) merged bottom-up:
    at each level the Morton code is shifted right until the level has about
    `target_degree` nodes per group; groups above 15 children are cut; finally
    single-child chains are collapsed."""
    from chroma.gpu import _native
    lib = _native.lib()
    vertices = np.ascontiguousarray(mesh.vertices, dtype=np.float32)
    triangles = np.ascontiguousarray(mesh.triangles, dtype=np.uint32)
    handle = ctypes.c_void_p()
    _native.check(lib.chr_bvh_build_grid(vertices.ctypes.data, len(vertices), triangles.ctypes.data,
                                         len(triangles), int(target_degree), ctypes.byref(handle)),
                  'chr_bvh_build_grid')
    try:
        nnodes, nlayers = ctypes.c_uint32(), ctypes.c_uint32()
        origin = np.zeros(3, dtype=np.float32)
        scale = ctypes.c_float()
        _native.check(lib.chr_bvh_result_info(handle, ctypes.byref(nnodes), ctypes.byref(nlayers),
                                              origin.ctypes.data, ctypes.byref(scale)), 'chr_bvh_result_info')
        nodes = np.empty(nnodes.value, dtype=uint4)
        layers = np.empty(nlayers.value, dtype=np.uint32)
        _native.check(lib.chr_bvh_result_copy(handle, nodes.ctypes.data, layers.ctypes.data),
                      'chr_bvh_result_copy')
    finally:
        lib.chr_bvh_result_free(handle)
    if verbose:
        print('BVH: %d nodes in %d layers' % (len(nodes), len(layers)))
    return BVH(WorldCoords(origin, np.float32(scale.value)), nodes, layers.astype(np.int64))
