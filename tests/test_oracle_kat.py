"""Pin the CPU oracle against the reference's own fixtures."""
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN
from film import film_rays
import oracle


def test_ray_intersection_kat(cube_geometry):
    """test/data/ray_intersection.npy: nearest-hit distances inside
    make.cube(1000).  The reference marks its own test stale (skip): its 56
    zero entries are edge rays an older intersect_triangle missed; every other
    ray must agree to float rounding (the reference ran with fast-math)."""
    from chroma.gpu.packing import PackedGeometry
    golden = np.load(os.path.join(GOLDEN, 'ray_intersection.npy'))
    pos, d = film_rays()
    dist, tri, _ = oracle.distance_to_mesh(PackedGeometry(cube_geometry), pos, d)
    hit = golden > 0
    assert (tri >= 0).all()
    rel = np.abs(dist[hit] - golden[hit]) / golden[hit]
    assert rel.max() < 1e-6
    assert (dist[hit] == golden[hit]).mean() > 0.6      # most are bit-identical
    assert (~hit).sum() == 56


def test_ray_intersection_analytic(cube_geometry):
    """From the cube centre every ray hits a face at 500/max|d_i|."""
    from chroma.gpu.packing import PackedGeometry
    from chroma import tools
    pos, d = tools.from_film()
    dist, tri, _ = oracle.distance_to_mesh(PackedGeometry(cube_geometry), pos, d)
    d32 = d.astype(np.float32)
    d32 /= np.linalg.norm(d32, axis=1)[:, None]
    expect = 500.0 / np.abs(d32).max(axis=1)
    assert (tri >= 0).all()
    assert np.max(np.abs(dist - expect) / expect) < 1e-6


def _rocrand_sequence_matrix():
    path = '/opt/rocm/include/rocrand/rocrand_xorwow_precomputed.h'
    if not os.path.exists(path):
        pytest.skip('rocRAND headers not installed')
    text = open(path).read()
    i = text.index('h_xorwow_sequence_jump_matrices')
    body = text[text.index('{', i):]
    nums = re.findall(r'(\d+)U?', body[:200000])
    return np.array([int(x) for x in nums[:800]], dtype=np.uint64).astype(np.uint32)


def test_xorwow_jump_matches_rocrand():
    """Our GF(2) construction of A^(2^67) (the cuRAND/rocRAND subsequence
    stride) equals rocRAND's precomputed sequence-jump matrix."""
    ref = _rocrand_sequence_matrix()
    ours = oracle.sequence_matrices(1)[0]
    assert np.array_equal(ours, ref)


def test_xorwow_recurrence_and_uniform():
    st = oracle.rng_init(4, seed=1234)
    u = oracle.uniforms(st.copy(), 4, 2, 1000)
    assert ((u > 0) & (u <= 1)).all()
    # restate the recurrence in numpy from the slot's state
    d, v = int(st[2]), [int(st[k * 4 + 2]) for k in range(1, 6)]
    out = []
    for _ in range(1000):
        t = (v[0] ^ (v[0] >> 2)) & 0xFFFFFFFF
        v = v[1:] + [((v[4] ^ ((v[4] << 4) & 0xFFFFFFFF)) ^ (t ^ ((t << 1) & 0xFFFFFFFF))) & 0xFFFFFFFF]
        d = (d + 362437) & 0xFFFFFFFF
        x = (v[4] + d) & 0xFFFFFFFF
        out.append(np.float32(np.float32(x) * np.float32(2.0 ** -32) + np.float32(2.0 ** -33)))
    assert np.array_equal(np.array(out, dtype=np.float32), u)


def test_xorwow_subsequences_differ():
    st = oracle.rng_init(64, seed=1)
    rows = st.reshape(6, 64)
    assert len({tuple(rows[:, s]) for s in range(64)}) == 64
    assert (rows[0] == rows[0, 0]).all()     # d is not moved by a 2^67 jump


def _first_uniforms(states, nslots):
    """The first curand_uniform of every slot, vectorised from the SoA states
    (d, v0..v4; chroma_rng.h chr_xorwow_next / chr_uniform01)."""
    st = states.reshape(6, nslots).astype(np.uint64)
    d, v0, v4 = st[0], st[1], st[5]
    m = np.uint64(0xFFFFFFFF)
    t = (v0 ^ (v0 >> np.uint64(2))) & m
    v4n = ((v4 ^ (v4 << np.uint64(4))) ^ (t ^ (t << np.uint64(1)))) & m
    x = (v4n + ((d + np.uint64(362437)) & m)) & m
    return (x.astype(np.float32) * np.float32(2.3283064365386963e-10) + np.float32(1.1641532182693481e-10))


def test_xorwow_seed0_pooled_ks_is_a_stream_property():
    """The reference's sample_cdf pin (test_sample_cdf.py: 128x128 slots,
    curand_init(0, slot, offset=rep), 50 reps) is judged on MI355X by per-rep
    KS uniformity plus a chi-square (tests/test_gpu_device_math.py), because
    the pooled continuous KS of its 819,200 draws is low at seed 0.  That low
    value belongs to the XORWOW stream itself, before any sampler: the first
    uniforms of the CPU restatement (oracle rng_init, the same generator the
    HIP path matches bit for bit) give the same p ~ 0.005 at seed 0 and
    unremarkable values at other seeds."""
    from scipy import stats
    n = 128 * 128

    def pooled(seed):
        u = np.concatenate([_first_uniforms(oracle.rng_init(n, seed=seed, offset=rep), n) for rep in range(50)])
        return stats.kstest(u.astype(np.float64), 'uniform').pvalue
    p0 = pooled(0)
    assert p0 < 0.02, p0
    assert all(pooled(s) > 0.05 for s in (1, 2)), [pooled(s) for s in (1, 2)]
    # the vectorised first draw is the generator's own
    st = oracle.rng_init(64, seed=0, offset=3)
    want = np.array([oracle.uniforms(st.copy(), 64, s, 1)[0] for s in range(64)], np.float32)
    assert np.array_equal(_first_uniforms(st, 64), want)
