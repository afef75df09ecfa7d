"""The lone walk split over two waves (walk_pair): on the same rays
it returns exactly walk_lone's nearest hit (record index; walk_lone is pinned to
the oracle through the tail parity tests, test_gpu_batches.py), with no lost
handshake or stack overflow, including flat (axis-parallel / plane-parallel)
directions and rays that start on a surface with their last hit excluded.
Reference walk semantics: chroma/cuda/mesh.h:45-126."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    from chroma.gpu import create_cuda_context
    return create_cuda_context()


def _rays(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-600.0, 600.0, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d[: n // 8, 2] = 0.0                       # plane-parallel
    d[n // 8: n // 4, 1:] = 0.0                # axis-parallel
    d /= np.linalg.norm(d, axis=1)[:, None]
    rays = np.zeros((n, 7), np.float32)
    rays[:, 0:3] = o
    rays[:, 3:6] = d.astype(np.float32)
    rays[:, 6] = np.full(n, -1, np.int32).view(np.float32)
    return rays


def _walk(det, rays, walker, nwaves, reps=2):
    import torch
    from chroma.gpu import _native, gpuarray as ga
    from chroma.gpu.tools import current_stream
    n = len(rays)
    dr = ga.to_gpu(rays.reshape(-1))
    out = ga.zeros(n * reps * 4 + 1, np.uint32)
    _native.call('chr_walk_lone_timing', det._handle, dr.gpudata, n, reps, nwaves, walker, out.gpudata,
                 current_stream())
    torch.cuda.synchronize()
    raw = out.get()
    return raw[:-1].reshape(n, reps, 4)[:, :, 0].astype(np.int32), int(raw[-1])


@pytest.mark.parametrize('nwaves', [1, 64])
def test_pair_walk_equals_lone(cuda, small_detector, nwaves):
    from chroma import gpu
    det = gpu.GPUDetector(small_detector)
    rays = _rays(512 if nwaves > 1 else 96, seed=3 + nwaves)
    lone, ov0 = _walk(det, rays, 0, nwaves)
    pair, ov1 = _walk(det, rays, 1, nwaves)
    assert ov0 == 0 and ov1 == 0
    assert np.array_equal(lone[:, 0], lone[:, 1]) and np.array_equal(pair[:, 0], pair[:, 1])
    assert np.array_equal(lone, pair)
    assert (lone[:, 0] >= 0).sum() > len(rays) // 2     # most rays hit something


def test_pair_walk_from_hits(cuda, small_detector, small_packed):
    """Rays with their nearest triangle excluded (last hit = that triangle's id, as a
    tail step's ray restarting on the surface it reached): the walk finds the next one."""
    from chroma import gpu
    from chroma.gpu import wide_bvh
    det = gpu.GPUDetector(small_detector)
    rec_id = np.asarray(wide_bvh.build(small_packed).rec_id)   # the same deterministic build as the upload's
    rays = _rays(512, seed=11)
    first, _ = _walk(det, rays, 0, 64, reps=1)
    hit = first[:, 0] >= 0
    rr = rays[hit].copy()
    rr[:, 6] = rec_id[first[hit, 0]].astype(np.int32).view(np.float32)
    lone, ov0 = _walk(det, rr, 0, 64)
    pair, ov1 = _walk(det, rr, 1, 64)
    assert ov0 == 0 and ov1 == 0 and np.array_equal(lone, pair)
    assert not np.array_equal(lone[:, 0], first[hit, 0])      # the excluded triangles are not found again
    assert np.all(lone[:, 0] != first[hit, 0])


def test_pair_walk_lost_handshake_recovers(cuda, small_detector):
    """a lost pair handshake must not return the tester's partial
    minimum.  walker 2 gives every handshake wait 2 polls, so handshakes are
    lost; the walker then walks the ray again alone and its workgroup pairs no
    more walks.  Every result equals walk_lone's, and the lost handshakes are
    counted (1 << 20 each), with no stack overflow."""
    from chroma import gpu
    det = gpu.GPUDetector(small_detector)
    rays = _rays(512, seed=17)
    lone, ov0 = _walk(det, rays, 0, 64)
    forced, ov2 = _walk(det, rays, 2, 64)
    assert ov0 == 0 and (ov2 & 0xFFFFF) == 0
    assert ov2 >> 20 >= 1                      # the recovery path ran
    assert np.array_equal(lone, forced)


def test_walk_up_equals_lone(cuda, small_detector, small_packed):
    """walk_up (the tail's lone walk started at the previous hit's leaf, climbing
    the ancestor chains in the node slots): from ANY start node it reaches every
    node once, so it returns walk_lone's record on every ray -- walker 3 starts
    ray r at node (r * 2654435761) mod nodes; walker 4 at the leaf of the ray's
    previous hit record (the tail's use), rays restarting on that surface."""
    from chroma import gpu
    from chroma.gpu import wide_bvh
    det = gpu.GPUDetector(small_detector)
    rays = _rays(512, seed=23)
    lone, ov0 = _walk(det, rays, 0, 64)
    up, ov3 = _walk(det, rays, 3, 64)
    seg, ov5 = _walk(det, rays, 5, 64)
    pre, ov7 = _walk(det, rays, 7, 64)
    assert ov0 == 0 and ov3 == 0 and ov5 == 0 and ov7 == 0
    assert np.array_equal(lone, up) and np.array_equal(lone, seg) and np.array_equal(lone, pre)
    # from the previous hit's leaf, that hit excluded
    rec_id = np.asarray(wide_bvh.build(small_packed).rec_id)
    first, _ = _walk(det, rays, 0, 64, reps=1)
    hit = first[:, 0] >= 0
    rr = np.zeros((int(hit.sum()), 8), np.float32)
    rr[:, :7] = rays[hit]
    rr[:, 6] = rec_id[first[hit, 0]].astype(np.int32).view(np.float32)
    rr[:, 7] = first[hit, 0].astype(np.int32).view(np.float32)
    lone2, _ = _walk(det, np.ascontiguousarray(rr[:, :7]), 0, 64)
    up2, ov4 = _walk(det, rr, 4, 64)
    assert ov4 == 0 and np.array_equal(lone2, up2)
    assert np.all(up2[:, 0] != first[hit, 0])      # the excluded triangles are not found again
