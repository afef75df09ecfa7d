"""Fixed-degree BVH (reference chroma/bvh/simple.py:5-28 + gpu/bvh.py:149-237
merge_nodes / bvh.cu make_parents).  Leaves are Morton ordered; each level
groups consecutive `degree` nodes under one parent.  The reference's optional
area-ratio re-parenting (max_ratio) is not reproduced: it only rearranges the
tree, it does not change which triangle a ray hits."""
import numpy as np

from chroma.bvh.bvh import BVH, CHILD_BITS, uint4


def _parents(children, degree):
    n = len(children)
    nparent = (n + degree - 1) // degree
    out = np.zeros(nparent, dtype=uint4)
    first = np.arange(nparent, dtype=np.uint64) * degree
    nchild = np.minimum(degree, n - first).astype(np.uint64)
    for axis in 'xyz':
        v = children[axis]
        lo = (v & 0xFFFF).astype(np.int64)
        hi = (v >> 16).astype(np.int64)
        pad = nparent * degree - n
        lo = np.concatenate([lo, np.full(pad, 1 << 20)]).reshape(nparent, degree).min(axis=1)
        hi = np.concatenate([hi, np.full(pad, -1)]).reshape(nparent, degree).max(axis=1)
        out[axis] = ((hi << 16) | lo).astype(np.uint32)
    out['w'] = ((nchild << np.uint64(CHILD_BITS)) | first).astype(np.uint32)
    return out


def make_simple_bvh(mesh, degree):
    from chroma.bvh.grid import make_recursive_grid_bvh
    if degree < 2 or degree > 15:
        raise ValueError('degree must be in [2, 15]')
    base = make_recursive_grid_bvh(mesh, target_degree=degree)   # for leaves + world coords
    leaves = base.nodes[base.layer_offsets[-1]:].copy()
    # Morton order of the leaves is the grid builder's leaf layer order
    layers = [leaves]
    while len(layers[0]) > 1:
        layers.insert(0, _parents(layers[0], degree))
    bounds = np.cumsum([0] + [len(l) for l in layers])
    nodes = np.concatenate(layers)
    for i in range(len(layers) - 1):   # child offsets: next layer start
        sl = slice(bounds[i], bounds[i + 1])
        w = nodes['w'][sl].astype(np.uint64)
        nchild = w >> np.uint64(CHILD_BITS)
        child = w & np.uint64((1 << CHILD_BITS) - 1)
        nodes['w'][sl] = ((nchild << np.uint64(CHILD_BITS)) | (child + np.uint64(bounds[i + 1]))).astype(np.uint32)
    return BVH(base.world_coords, nodes, bounds[:-1])
