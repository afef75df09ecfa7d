"""The traversal BVH (csrc/wide_bvh.cpp) on the host: structure only.

What the kernel's result equivalence rests on (wide_bvh.cpp header):
  * every triangle reachable in the reference BVH appears exactly once, with
    its reference leaf-node words and its rank in the reference DFS order
    (mesh.h:75-117: a group's leaves in index order, then its inner children's
    subtrees, last pushed first);
  * every child box, decoded exactly as the kernel decodes it
    (fmaf(q, 2^(e-127), origin)), contains the reference leaf boxes of every
    triangle below it;
  * triangle records carry the float32 Moller-Trumbore operands.
The walk itself is checked against the oracle on the GPU (test_gpu_parity.py).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _fma32(q, s, o):
    """float32 fmaf(q, s, o) for small-integer q (exact in long double, one rounding)."""
    return (np.asarray(q, np.longdouble) * np.asarray(s, np.longdouble) + np.asarray(o, np.longdouble)).astype(np.float32)


def _reference_dfs(nodes):
    """(rank, leaf words) per triangle from the reference node array."""
    w = nodes[:, 3]
    ntri_guess = int((w[(w >> 28) == 0] & 0x0FFFFFFF).max()) + 1
    rank = np.full(ntri_guess, -1, dtype=np.int64)
    leaf = np.zeros((ntri_guess, 3), dtype=np.uint32)
    r = 0
    if (w[0] >> 28) == 0:
        t = int(w[0] & 0x0FFFFFFF)
        rank[t] = 0
        leaf[t] = nodes[0, :3]
        return rank, leaf
    stack = [int(w[0])]
    while stack:
        ww = stack.pop()
        first, n = ww & 0x0FFFFFFF, ww >> 28
        for i in range(first, first + n):
            wi = int(w[i])
            if (wi >> 28) == 0:
                t = wi & 0x0FFFFFFF
                if rank[t] < 0:
                    rank[t] = r
                    leaf[t] = nodes[i, :3]
                    r += 1
            else:
                stack.append(wi)
    return rank, leaf


def _check(packed):
    from chroma.bvh.wide import build_wide_bvh, WIDE_INNER
    wb = build_wide_bvh(packed)
    assert wb.usable
    nodes, tris = wb.nodes, wb.tris
    ntri = len(packed.triangles)
    # exactly once each, with reference rank and leaf words
    assert len(tris) == ntri
    assert np.array_equal(np.sort(tris['id']), np.arange(ntri))
    rank, leaf = _reference_dfs(packed.nodes)
    assert np.array_equal(tris['rank'], rank[tris['id']])
    assert np.array_equal(tris['leaf'], leaf[tris['id']])
    # the triangle's own float vertices (edges and normal formed in the kernels)
    v = packed.vertices[packed.triangles[tris['id']]]
    assert np.array_equal(tris['v0'], v[:, 0])
    assert np.array_equal(tris['v1'], v[:, 1])
    assert np.array_equal(tris['v2'], v[:, 2])
    assert np.array_equal(tris['code'], np.asarray(packed.material_codes, np.uint32)[tris['id']])
    # reference leaf boxes (decoded as the reference does)
    q = tris['leaf']
    tlo = _fma32(q & 0xFFFF, packed.world_scale, packed.world_origin[None, :])
    thi = _fma32(q >> 16, packed.world_scale, packed.world_origin[None, :])
    # subtree unions bottom-up: inner children always have larger indices
    nlo = np.full((len(nodes), 3), np.inf, np.float32)
    nhi = np.full((len(nodes), 3), -np.inf, np.float32)
    scale = ((nodes['exp'].astype(np.uint32) << 23)).view(np.float32)
    tested = 0
    for i in range(len(nodes) - 1, -1, -1):
        nd = nodes[i]
        assert 1 <= nd['nchild'] <= 8
        kinds = nd['kind']
        assert (kinds[:nd['nchild']] != 0).all() and (kinds[nd['nchild']:] == 0).all()
        for k in range(nd['nchild']):
            clo = _fma32(nd['qlo'][:, k], scale[i], nd['origin'])
            chi = _fma32(nd['qhi'][:, k], scale[i], nd['origin'])
            if kinds[k] == WIDE_INNER:
                c = nd['child_base'] + nd['off'][k]
                assert c > i
                slo, shi = nlo[c], nhi[c]
            else:
                assert 1 <= kinds[k] <= 4
                a = nd['tri_base'] + nd['off'][k]
                slo, shi = tlo[a:a + kinds[k]].min(0), thi[a:a + kinds[k]].max(0)
                tested += int(kinds[k])
            assert (clo <= slo).all() and (chi >= shi).all(), 'node %d child %d box does not contain its subtree' % (i, k)
            nlo[i] = np.minimum(nlo[i], slo)
            nhi[i] = np.maximum(nhi[i], shi)
    assert tested == ntri
    return wb


def test_wide_bvh_small_detector(small_packed):
    wb = _check(small_packed)
    assert wb.max_depth <= 12
    # an 8-wide tree with <=4-triangle leaves is far smaller than the reference one
    assert len(wb.nodes) < len(small_packed.nodes) / 4


def test_wide_bvh_cube(cube_geometry):
    from chroma.gpu.packing import PackedGeometry
    _check(PackedGeometry(cube_geometry))


def test_wide_bvh_physics_scene():
    import scenes
    from chroma import loader
    from chroma.gpu.packing import PackedGeometry
    _check(PackedGeometry(loader.create_geometry_from_obj(scenes.physics_scene())))


@pytest.mark.parametrize('ntri', [1, 3, 5, 9])
def test_wide_bvh_tiny_meshes(ntri):
    """Root-is-leaf and few-triangle edge cases."""
    from chroma.geometry import Mesh, Solid, Geometry
    from chroma.demo.optics import water
    from chroma.gpu.packing import PackedGeometry
    from chroma import loader
    rng = np.random.RandomState(ntri)
    v = rng.uniform(-100, 100, size=(3 * ntri, 3)).astype(np.float32)
    t = np.arange(3 * ntri, dtype=np.int32).reshape(-1, 3)
    g = Geometry(water)
    g.add_solid(Solid(Mesh(v, t, round=False, remove_null_triangles=False), water, water))
    _check(PackedGeometry(loader.create_geometry_from_obj(g)))
