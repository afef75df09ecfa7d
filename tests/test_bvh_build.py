"""BVH: the product's C++ builder vs the numpy restatement of the reference
builder (oracle/bvh_ref.py), and the reference's node-packing KAT
(test/test_bvh.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
import bvh_ref


@pytest.mark.parametrize('name', ['lionsolid', 'detector_small', 'cube_1000', 'pmt_lc_solid'])
def test_grid_bvh_matches_restatement(name):
    from chroma.bvh import make_recursive_grid_bvh
    from chroma.geometry import Mesh
    d = np.load(os.path.join(GOLDEN, name + '.npz'))
    mesh = Mesh(d['vertices'], d['triangles'], round=False, remove_null_triangles=False)
    b = make_recursive_grid_bvh(mesh, target_degree=3)
    origin, scale, nodes, bounds = bvh_ref.make_recursive_grid_bvh(mesh.vertices, mesh.triangles.astype(np.uint32))
    assert np.array_equal(b.nodes, nodes)
    assert np.array_equal(np.asarray(b.layer_offsets), bounds)
    assert np.array_equal(b.world_coords.world_origin, origin) and b.world_coords.world_scale == scale


@pytest.mark.parametrize('degree', [2, 3, 4])
def test_bvh_invariants(degree):
    """Every inner node's box contains its children; each triangle is
    reachable exactly once (test_bvh_simple.py checks degrees 2/3/4)."""
    from chroma.bvh import make_recursive_grid_bvh, unpack_nodes, BVH
    from chroma.geometry import Mesh
    d = np.load(os.path.join(GOLDEN, 'lionsolid.npz'))
    b = make_recursive_grid_bvh(Mesh(d['vertices'], d['triangles']), target_degree=degree)
    assert isinstance(b, BVH)
    u = unpack_nodes(b.nodes)
    seen = np.zeros(len(d['triangles']), dtype=int)
    stack = [0]
    while stack:
        i = stack.pop()
        if u['nchild'][i] == 0:
            seen[int(u['child'][i])] += 1
            continue
        c0, n = int(u['child'][i]), int(u['nchild'][i])
        assert 2 <= n <= 15
        for c in range(c0, c0 + n):
            for a in 'xyz':
                assert u[a + 'lo'][c] >= u[a + 'lo'][i] and u[a + 'hi'][c] <= u[a + 'hi'][i]
            stack.append(c)
    assert (seen == 1).all()


def test_simple_bvh_is_bvh():
    from chroma.bvh import make_simple_bvh, BVH, unpack_nodes
    from chroma.geometry import Mesh
    d = np.load(os.path.join(GOLDEN, 'lionsolid.npz'))
    for degree in (2, 3, 4):
        b = make_simple_bvh(Mesh(d['vertices'], d['triangles']), degree)
        assert isinstance(b, BVH)
        assert unpack_nodes(b.nodes[:1])['nchild'][0] <= degree


# ---- reference test/test_bvh.py KAT: world coords and a hand-built binary tree
def test_world_coords():
    from chroma.bvh import WorldCoords, OutOfRangeError
    c = WorldCoords([-1, -1, -1], 0.1)
    np.testing.assert_array_max_ulp(c.fixed_to_world([0, 1, 100]), [-1.0, -0.9, 9.0], dtype=np.float32)
    np.testing.assert_array_equal(c.world_to_fixed([-1.0, -0.9, 9.0]), [0, 1, 100])
    np.testing.assert_array_equal(c.world_to_fixed([[1.0, 3.0, 5.0], [20.0, 30.0, 40.0]]),
                                  [[20, 40, 60], [210, 310, 410]])
    with pytest.raises(OutOfRangeError):
        c.world_to_fixed([-2.0, 0.0, 0.0])
    with pytest.raises(OutOfRangeError):
        c.world_to_fixed([0.0, 1e9, 0.0])


def _kat_bvh():
    from chroma.bvh import BVH, WorldCoords, uint4, CHILD_BITS
    nodes = np.empty(7, dtype=uint4)
    # layer 0: root with 2 children at 1; layer 1: two nodes, children at 3 and 5; layer 2: leaves
    boxes = [((0, 10), (0, 10), (0, 10)), ((0, 5), (0, 10), (0, 10)), ((5, 10), (0, 10), (0, 10)),
             ((0, 5), (0, 5), (0, 10)), ((0, 5), (5, 10), (0, 10)), ((5, 10), (0, 5), (0, 10)),
             ((5, 10), (5, 10), (0, 10))]
    for i, (bx, by, bz) in enumerate(boxes):
        nodes['x'][i] = bx[1] << 16 | bx[0]
        nodes['y'][i] = by[1] << 16 | by[0]
        nodes['z'][i] = bz[1] << 16 | bz[0]
    nodes['w'] = [2 << CHILD_BITS | 1, 2 << CHILD_BITS | 3, 2 << CHILD_BITS | 5, 0, 1, 2, 3]
    return BVH(WorldCoords(np.array([-1.0, -1.0, -1.0]), 0.1), nodes, [0, 1, 3])


def test_unpack_and_layers():
    from chroma.bvh import unpack_nodes
    b = _kat_bvh()
    u = unpack_nodes(b.nodes)
    assert list(u['nchild']) == [2, 2, 2, 0, 0, 0, 0]
    assert list(u['child']) == [1, 3, 5, 0, 1, 2, 3]
    assert list(u['xhi'][:3]) == [10, 5, 10]
    assert b.layer_count() == 3 and len(b) == 7
    assert len(b.get_layer(0)) == 1 and len(b.get_layer(1)) == 2 and len(b.get_layer(2)) == 4
    # layer areas in fixed units: 2*(10*10*3)=600 root; leaves 2*(25+50+50)=250 each
    assert b.get_layer(0).area_fixed() == 600.0
    assert b.get_layer(2).area_fixed() == 4 * 250.0
    np.testing.assert_allclose(b.get_layer(0).area(), 600.0 * 0.01, rtol=1e-6)
    lo, hi = b.get_layer(1).get_bounds()
    np.testing.assert_allclose(lo[0], [-1, -1, -1]) and np.testing.assert_allclose(hi[1], [0.0, 0.0, 0.0], atol=1e-6)
