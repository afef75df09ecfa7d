"""Host view of the traversal BVH the gfx950 kernel walks (csrc/wide_bvh.h).

GPUGeometry obtains this tree through chroma.gpu.wide_bvh (cached compact
form, or a build); this module exposes the full build, records included, so
tests can check its invariants (containment after the kernel's float decode,
every reachable triangle exactly once, reference DFS ranks).
No reference counterpart: it is derived from the reference BVH
(chroma/bvh/grid.py) and never replaces it in the Python API.
"""
import ctypes

import numpy as np

from chroma.gpu import _native

WIDE_INNER = 0x80

wide_node_dtype = np.dtype([('origin', '<f4', 3), ('exp', 'u1', 3), ('nchild', 'u1'),
                            ('qlo', 'u1', (3, 8)), ('qhi', 'u1', (3, 8)),
                            ('child_base', '<u4'), ('tri_base', '<u4'),
                            ('kind', 'u1', 8), ('off', 'u1', 8), ('pad', '<u4', 2)])
wide_tri_dtype = np.dtype([('v0', '<f4', 3), ('v1', '<f4', 3), ('v2', '<f4', 3), ('id', '<u4'),
                           ('rank', '<u4'), ('leaf', '<u4', 3), ('code', '<u4'), ('pad', '<u4')])
assert wide_node_dtype.itemsize == 96 and wide_tri_dtype.itemsize == 64


class WideBVH(object):
    def __init__(self, nodes, tris, max_depth, usable):
        self.nodes, self.tris, self.max_depth, self.usable = nodes, tris, max_depth, usable


def build_wide_bvh(packed):
    """packed: chroma.gpu.packing.PackedGeometry."""
    h = ctypes.c_void_p()
    _native.call('chr_wide_bvh_build', ctypes.byref(packed.desc()), ctypes.byref(h))
    try:
        nn, nt, depth, usable = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int32()
        _native.call('chr_wide_bvh_info', h, ctypes.byref(nn), ctypes.byref(nt), ctypes.byref(depth),
                     ctypes.byref(usable))
        nodes = np.zeros(nn.value, dtype=wide_node_dtype)
        tris = np.zeros(nt.value, dtype=wide_tri_dtype)
        _native.call('chr_wide_bvh_copy', h, nodes.ctypes.data, tris.ctypes.data)
    finally:
        _native.call('chr_wide_bvh_free', h)
    return WideBVH(nodes, tris, depth.value, bool(usable.value))
