"""chr_propagate_batches (chroma.gpu.propagate_batches): several photon
batches propagated with one rng_states, batch i's multi-step tail on a second
stream while batch i+1 starts.  The contract is bit-identity with the same
GPUPhotons.propagate calls made one after the other (the event loop of the
reference Simulation, sim.py:116-160): every photon array and every RNG slot
state, plus the oracle run sequentially on the small detector.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

FIELDS = ('pos', 'dir', 'pol', 'wavelengths', 't', 'flags', 'last_hit_triangles', 'weights')


@pytest.fixture(scope='module')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    torch.cuda.set_device(0)


def _sources(sizes, seed):
    from chroma.photon_source import isotropic
    return [isotropic(n, seed=seed + i) if n else None for i, n in enumerate(sizes)]


def _gpu_photons(src):
    from chroma import gpu
    return gpu.GPUPhotons(src, copy_flags=True, copy_triangles=False, copy_weights=False)


def _run(det, sources, ntpb, max_blocks, max_steps, batched, seed=3):
    from chroma import gpu
    rng = gpu.get_rng_states(ntpb * max_blocks, seed=seed)
    gps = [_gpu_photons(s) for s in sources if s is not None]
    if batched:
        stats = gpu.propagate_batches(gps, det, rng, nthreads_per_block=ntpb, max_blocks=max_blocks,
                                      max_steps=max_steps)
    else:
        stats = []
        for gp in gps:
            gp.propagate(det, rng, nthreads_per_block=ntpb, max_blocks=max_blocks, max_steps=max_steps)
            stats.append(gp.last_stats)
    return [gp.get() for gp in gps], rng.get(), stats


def _same(a, b, label):
    for f in FIELDS:
        assert np.array_equal(getattr(a, f), getattr(b, f)), '%s: %s differs' % (label, f)


@pytest.mark.parametrize('ntpb,max_blocks', [(64, 64), (256, 64), (64, 256)])
def test_batches_equal_sequential_and_oracle(cuda, small_detector, small_packed, ntpb, max_blocks):
    """Batches of 30k / 70k / 5k / 120k photons (one-step slots, then tails of
    < ntpb*128 photons) on the 2-PMT detector: batched == sequential GPU ==
    sequential oracle, photons and RNG states."""
    from chroma import gpu
    det = gpu.GPUDetector(small_detector)
    sources = _sources([30000, 70000, 5000, 120000], seed=11)
    seq, rng_seq, st_seq = _run(det, sources, ntpb, max_blocks, 1000, batched=False)
    bat, rng_bat, st_bat = _run(det, sources, ntpb, max_blocks, 1000, batched=True)
    for i, (a, b) in enumerate(zip(bat, seq)):
        _same(a, b, 'batch %d' % i)
    assert np.array_equal(rng_bat, rng_seq)
    for sa, sb in zip(st_bat, st_seq):
        assert sa.steps_run == sb.steps_run and sa.tail_photons == sb.tail_photons
        assert sa.trace_rays == sb.trace_rays and sa.stack_overflows == 0
    assert sum(s.tail_photons for s in st_bat) > 0     # tails ran (on the tail stream)
    nslots = ntpb * max_blocks
    states = oracle.rng_init(nslots, seed=3)
    for i, src in enumerate(sources):
        host = oracle.HostPhotons(src)
        host.last_hit_triangles[:] = -1
        host.weights[:] = 1.0
        oracle.propagate(small_packed, host, states, nslots, ntpb, max_blocks, 1000)
        for f in ('flags', 'last_hit_triangles'):
            assert np.array_equal(getattr(bat[i], f), getattr(host, f)), 'oracle batch %d: %s' % (i, f)
        for f in ('pos', 'dir', 'pol', 't', 'wavelengths'):
            a = getattr(bat[i], f).astype(np.float64)
            b = getattr(host, f).astype(np.float64)
            assert np.all(np.abs(a - b) <= 1e-5 * np.maximum(np.abs(b), 1.0)), 'oracle batch %d: %s' % (i, f)
    assert np.array_equal(rng_bat, states.reshape(6, nslots))


@pytest.mark.parametrize('pattern', ['aa', 'aba', 'abcdeb'])
def test_batches_shared_photons(cuda, small_detector, pattern):
    """Batches listing the same GPUPhotons more than once (aliasing arrays: a
    batch waits for the earlier one it shares photons with, also when that one
    is two batches back) and more batches than buffer contexts == the same
    propagate calls in order."""
    from chroma import gpu
    det = gpu.GPUDetector(small_detector)
    names = sorted(set(pattern))
    src = dict(zip(names, _sources([40000 + 7000 * i for i in range(len(names))], seed=5)))
    out = {}
    for batched in (False, True):
        rng = gpu.get_rng_states(64 * 64, seed=9)
        gps = {k: _gpu_photons(src[k]) for k in names}
        seq = [gps[k] for k in pattern]
        if batched:
            gpu.propagate_batches(seq, det, rng, nthreads_per_block=64, max_blocks=64, max_steps=7)
        else:
            for gp in seq:
                gp.propagate(det, rng, nthreads_per_block=64, max_blocks=64, max_steps=7)
        out[batched] = ({k: gps[k].get() for k in names}, rng.get())
    for k in names:
        _same(out[True][0][k], out[False][0][k], '%s:%s' % (pattern, k))
    assert np.array_equal(out[True][1], out[False][1])


def test_batches_with_copies_and_weights(cuda, small_detector):
    """Batches of GPUPhotons with ncopies > 1 (clones interleaved in the queue,
    photon.py:242-250), and use_weights (every slot a multi-step tail) ==
    the same propagate calls in order."""
    from chroma import gpu
    det = gpu.GPUDetector(small_detector)
    srcs = _sources([12000, 9000, 15000], seed=31)
    for use_weights, copies in ((False, (3, 1, 2)), (True, (1, 2, 1))):
        out = {}
        for batched in (False, True):
            rng = gpu.get_rng_states(64 * 64, seed=4)
            gps = [gpu.GPUPhotons(s, ncopies=c, copy_flags=True, copy_triangles=False, copy_weights=False)
                   for s, c in zip(srcs, copies)]
            kw = dict(nthreads_per_block=64, max_blocks=64, max_steps=40, use_weights=use_weights)
            if batched:
                gpu.propagate_batches(gps, det, rng, **kw)
            else:
                for gp in gps:
                    gp.propagate(det, rng, **kw)
            out[batched] = ([gp.get() for gp in gps], rng.get())
        for i, (a, b) in enumerate(zip(out[True][0], out[False][0])):
            _same(a, b, 'weights=%s batch %d' % (use_weights, i))
        assert np.array_equal(out[True][1], out[False][1])


def test_batches_empty_and_single(cuda, small_detector):
    """Empty batches are skipped; one batch is one chr_propagate."""
    from chroma import gpu
    det = gpu.GPUDetector(small_detector)
    rng = gpu.get_rng_states(64 * 64, seed=2)
    assert gpu.propagate_batches([], det, rng, nthreads_per_block=64, max_blocks=64) == []
    src = _sources([20000], seed=8)[0]
    a, b = _gpu_photons(src), _gpu_photons(src)
    r1, r2 = gpu.get_rng_states(64 * 64, seed=2), gpu.get_rng_states(64 * 64, seed=2)
    gpu.propagate_batches([a], det, r1, nthreads_per_block=64, max_blocks=64, max_steps=50)
    b.propagate(det, r2, nthreads_per_block=64, max_blocks=64, max_steps=50)
    _same(a.get(), b.get(), 'single')
    assert np.array_equal(r1.get(), r2.get())


@pytest.fixture(scope='module')
def tiny_geo():
    from chroma import demo, loader
    return loader.create_geometry_from_obj(demo.tiny())


@pytest.mark.timeout(600)
def test_batches_c2_scale(cuda, tiny_geo):
    """Three 2^20-photon batches on demo.tiny() with the bench launch shape
    (512 x 1024): binned first steps overlapping the previous tail; batched ==
    sequential, photons and RNG states."""
    from chroma import gpu
    det = gpu.GPUDetector(tiny_geo)
    sources = _sources([1 << 20, 1 << 20, 1 << 20], seed=20260102)
    seq, rng_seq, _ = _run(det, sources, 512, 1024, 1000, batched=False)
    bat, rng_bat, st = _run(det, sources, 512, 1024, 1000, batched=True)
    for i, (a, b) in enumerate(zip(bat, seq)):
        _same(a, b, 'C2 batch %d' % i)
    assert np.array_equal(rng_bat, rng_seq)
    assert all(s.trace_launches >= 1 and s.tail_photons > 0 for s in st)


def test_max_steps_zero_and_negative(cuda, small_detector):
    """max_steps=0 runs no launch (the reference's `while step < max_steps`
    loop, photon.py:255) on both the sequential and the batched entry point:
    photons and RNG states untouched.  A negative max_steps is rejected before
    any device work (it would size the slot-control words)."""
    from chroma import gpu
    from chroma.gpu import _native
    det = gpu.GPUDetector(small_detector)
    src = _sources([3000, 2000], seed=41)
    gps = [_gpu_photons(s) for s in src]
    before = [gp.get() for gp in gps]
    rng = gpu.get_rng_states(64 * 64, seed=6)
    rng0 = rng.get()
    gps[0].propagate(det, rng, nthreads_per_block=64, max_blocks=64, max_steps=0)
    assert gps[0].last_stats.steps_run == 0 and gps[0].last_stats.final_alive == 3000
    st = gpu.propagate_batches(gps, det, rng, nthreads_per_block=64, max_blocks=64, max_steps=0)
    assert [s.steps_run for s in st] == [0, 0] and [s.final_alive for s in st] == [3000, 2000]
    for a, b in zip(gps, before):
        _same(a.get(), b, 'max_steps=0')
    assert np.array_equal(rng.get(), rng0)
    for call in (lambda: gps[0].propagate(det, rng, nthreads_per_block=64, max_blocks=64, max_steps=-1),
                 lambda: gpu.propagate_batches(gps, det, rng, nthreads_per_block=64, max_blocks=64, max_steps=-3)):
        with pytest.raises(_native.NativeError, match='max_steps'):
            call()
    assert np.array_equal(rng.get(), rng0)


def test_batches_slot_timing_modes_identical(cuda, small_detector, monkeypatch):
    """The tail stream's dependency on a slot: its trace-start event by default,
    the end of the slot's one-step kernels with every slot event recorded
    (CHR_SLOT_TIMING=1).  Every kernel of a tail-mode slot on the caller's
    stream exits at once, so both give the same photons and RNG states."""
    from chroma import gpu
    det = gpu.GPUDetector(small_detector)
    sources = _sources([30000, 70000, 5000, 120000], seed=17)
    out = {}
    for mode in ('t', '0', '1'):    # the default (trace launch pairs), none, every slot event
        monkeypatch.setenv('CHR_SLOT_TIMING', mode)
        out[mode] = _run(det, sources, 64, 256, 1000, batched=True)
    for mode in ('0', '1'):
        for i, (a, b) in enumerate(zip(out['t'][0], out[mode][0])):
            _same(a, b, 'CHR_SLOT_TIMING=%s batch %d' % (mode, i))
        assert np.array_equal(out['t'][1], out[mode][1])
    assert sum(s.tail_photons for s in out['t'][2]) > 0


# Every run-time switch the library reads (include/chroma_amd.h lists them)
# gives the same photons and RNG states as the default, sequential and batched:
#   CHR_HOST_STEPS=1        the host reads the survivor count every step
#   CHR_STEP_LAUNCH=0       one launch per chunk (the reference's launch structure)
#   CHR_TRACE_STEPS=1       per-step stderr lines (debugging)
#   CHR_PROPAGATE_VARIANT   2/4 fused step kernels, 7/8 binning every / no step, 1 the
#                           exact-order walk of the reference BVH, 5 the counting form
#   CHR_PAIR_WALK=0         the tail's lone walks without a tester wave (walk_lone)
#   CHR_WALK_UP=0 / 2 / 4   the tail's walks from the root / only its lone walks climbing / no chain prefetch
#   CHR_SLOT_TIMING         test_batches_slot_timing_modes_identical
#   CHR_WIDE_LEAF_MAX / CHR_EXACT_ORDER_ONLY: test_geometry_build_switches_identical
SWITCHES = [('CHR_HOST_STEPS', '1'), ('CHR_STEP_LAUNCH', '0'), ('CHR_TRACE_STEPS', '1'),
            ('CHR_PROPAGATE_VARIANT', '2'), ('CHR_PROPAGATE_VARIANT', '4'), ('CHR_PROPAGATE_VARIANT', '7'),
            ('CHR_PROPAGATE_VARIANT', '8'), ('CHR_PROPAGATE_VARIANT', '1'), ('CHR_PROPAGATE_VARIANT', '5'),
            ('CHR_PAIR_WALK', '0'), ('CHR_WALK_UP', '0'), ('CHR_WALK_UP', '2'), ('CHR_WALK_UP', '4')]


@pytest.mark.parametrize('switch,value', SWITCHES)
def test_switches_identical(cuda, small_detector, monkeypatch, switch, value):
    sources = _sources([30000, 70000, 5000, 120000], seed=29)
    from chroma import gpu
    det = gpu.GPUDetector(small_detector)
    monkeypatch.delenv(switch, raising=False)
    base = {b: _run(det, sources, 64, 256, 1000, batched=b) for b in (False, True)}
    monkeypatch.setenv(switch, value)
    for batched in (False, True):
        alt = _run(det, sources, 64, 256, 1000, batched=batched)
        for i, (a, b) in enumerate(zip(base[batched][0], alt[0])):
            _same(a, b, '%s=%s batched=%s batch %d' % (switch, value, batched, i))
        assert np.array_equal(base[batched][1], alt[1])
    assert sum(s.tail_photons for s in base[True][2]) > 0
    assert sum(s.trace_launches for s in base[True][2]) > 0


@pytest.mark.parametrize('switch,value', [('CHR_WIDE_LEAF_MAX', '4'), ('CHR_WIDE_LEAF_MAX', '1'),
                                          ('CHR_EXACT_ORDER_ONLY', '1')])
def test_geometry_build_switches_identical(cuda, small_detector, monkeypatch, switch, value):
    """The traversal BVH's leaf size (a build-time setting, part of its cache key)
    and the exact-order walk only (no traversal BVH uploaded): same photons."""
    import copy
    from chroma import gpu
    sources = _sources([30000, 70000], seed=37)
    base = _run(gpu.GPUDetector(small_detector), sources, 64, 256, 1000, batched=True)
    monkeypatch.setenv(switch, value)
    geo = copy.copy(small_detector)
    geo.bvh = copy.copy(small_detector.bvh)
    geo.bvh.wide = None
    det = gpu.GPUDetector(geo)
    alt = _run(det, sources, 64, 256, 1000, batched=True)
    for i, (a, b) in enumerate(zip(base[0], alt[0])):
        _same(a, b, '%s=%s batch %d' % (switch, value, i))
    assert np.array_equal(base[1], alt[1])


def test_mirror_scene_long_tail_parity(cuda):
    """The physics scene (97% specular mirror plate, wire planes, every surface
    model) at 4000 photons over 64 x 64 slots, 1000 steps: every step after the
    first runs in the tail kernel, whose waves thin out to a few walking photons
    (walk_lone for one, the segment walk for several).  HIP == oracle."""
    import scenes
    from chroma import gpu, loader
    from chroma.gpu.packing import PackedGeometry
    geo = loader.create_geometry_from_obj(scenes.physics_scene())
    det = gpu.GPUDetector(geo)
    src = scenes.photon_sources(4000, seed=41)
    got, rng, stats = _run(det, [src], 64, 64, 1000, batched=False, seed=5)
    nslots = 64 * 64
    states = oracle.rng_init(nslots, seed=5)
    host = oracle.HostPhotons(src)
    host.last_hit_triangles[:] = -1
    host.weights[:] = 1.0
    oracle.propagate(PackedGeometry(geo), host, states, nslots, 64, 64, 1000)
    for f in ('flags', 'last_hit_triangles'):
        assert np.array_equal(getattr(got[0], f), getattr(host, f)), 'mirror scene: %s' % f
    for f in ('pos', 'dir', 'pol', 't', 'wavelengths'):
        a = getattr(got[0], f).astype(np.float64)
        b = getattr(host, f).astype(np.float64)
        assert np.all(np.abs(a - b) <= 1e-5 * np.maximum(np.abs(b), 1.0)), 'mirror scene: %s' % f
    assert np.array_equal(rng, states.reshape(6, nslots))
    assert stats[0].tail_photons > 0
    if stats[0].tail_long_steps > 0:   # long-lived photons walk with a tester wave (walk_pair)
        assert stats[0].tail_long_paired_steps > 0
