"""Packed BVH node array + fixed-point world coordinates
(reference chroma/bvh/bvh.py:11-195).

A node is a uint4 record: x, y, z hold the quantised box (low 16 bits: lower
bound, high 16 bits: upper bound) and w = nchild << CHILD_BITS | child.  Inner
nodes point at `nchild` contiguous children; leaves (nchild == 0) hold a
triangle index.  World position = world_origin + fixed * world_scale.
"""
import numpy as np

uint4 = np.dtype([('x', '<u4'), ('y', '<u4'), ('z', '<u4'), ('w', '<u4')])

CHILD_BITS = 28
NCHILD_MASK = np.uint64(0xFFFF << CHILD_BITS)

__all__ = ['uint4', 'CHILD_BITS', 'NCHILD_MASK', 'unpack_nodes', 'OutOfRangeError', 'WorldCoords', 'BVH',
           'BVHLayerSlice', 'node_areas']


def unpack_nodes(nodes):
    """Record array with xlo/xhi/ylo/yhi/zlo/zhi (uint16), child (uint64),
    nchild (uint16) for each packed node."""
    out = np.empty(len(nodes), dtype=[('xlo', np.uint16), ('xhi', np.uint16), ('ylo', np.uint16),
                                      ('yhi', np.uint16), ('zlo', np.uint16), ('zhi', np.uint16),
                                      ('child', np.uint64), ('nchild', np.uint16)])
    for axis in 'xyz':
        out[axis + 'lo'] = nodes[axis] & 0xFFFF
        out[axis + 'hi'] = nodes[axis] >> 16
    w = nodes['w'].astype(np.uint64)
    out['child'] = w & ~NCHILD_MASK
    out['nchild'] = w >> np.uint64(CHILD_BITS)
    return out


class OutOfRangeError(Exception):
    """World coordinates outside the 16-bit fixed point range."""


class WorldCoords(object):
    """world = world_origin + fixed * world_scale (16-bit unsigned fixed)."""
    MAX_INT = 2 ** 16 - 1

    def __init__(self, world_origin, world_scale):
        self.world_origin = np.array(world_origin, dtype=np.float32)
        self.world_scale = np.float32(world_scale)

    def world_to_fixed(self, world):
        fixed = ((np.asarray(world, dtype=np.float64) - self.world_origin) / self.world_scale).round()
        if int(fixed.max()) > WorldCoords.MAX_INT or fixed.min() < 0:
            raise OutOfRangeError('range = (%f, %f)' % (fixed.min(), fixed.max()))
        return fixed.astype(np.uint16)

    def fixed_to_world(self, fixed):
        return np.asarray(fixed) * self.world_scale + self.world_origin


def node_areas(nodes):
    """Surface area of each node's box, fixed-point units."""
    u = unpack_nodes(nodes)
    d = [u[a + 'hi'].astype(float) - u[a + 'lo'] for a in 'xyz']
    return 2.0 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0])


class BVH(object):
    """Nodes (root first, layers contiguous in depth order) + layer offsets."""

    def __init__(self, world_coords, nodes, layer_offsets):
        self.world_coords = world_coords
        self.nodes = nodes
        self.layer_offsets = list(layer_offsets)
        self.layer_bounds = list(layer_offsets) + [len(nodes)]

    def get_layer(self, layer_number):
        sl = slice(self.layer_bounds[layer_number], self.layer_bounds[layer_number + 1])
        return BVHLayerSlice(world_coords=self.world_coords, nodes=self.nodes[sl])

    def layer_count(self):
        return len(self.layer_offsets)

    def __len__(self):
        return len(self.nodes)


class BVHLayerSlice(object):
    """One layer of a BVH (a view: edits change the parent's nodes)."""

    def __init__(self, world_coords, nodes):
        self.world_coords = world_coords
        self.nodes = nodes

    def __len__(self):
        return len(self.nodes)

    def areas_fixed(self):
        return node_areas(self.nodes)

    def area_fixed(self):
        return node_areas(self.nodes).sum()

    def area(self):
        return self.area_fixed().sum() * self.world_coords.world_scale ** 2

    def get_bounds(self):
        u = unpack_nodes(self.nodes)
        lo = np.dstack([u[s] for s in ('xlo', 'ylo', 'zlo')]).squeeze()
        hi = np.dstack([u[s] for s in ('xhi', 'yhi', 'zhi')]).squeeze()
        return (np.atleast_2d(self.world_coords.fixed_to_world(lo)),
                np.atleast_2d(self.world_coords.fixed_to_world(hi)))
