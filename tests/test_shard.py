"""Photon-sharded multi-GPU plumbing (chroma.gpu.shard) on CPU with the gloo
backend, world size 2: slicing, the rank-ordered hit gather, the hit record
packing, and the DAQ channel reduction (unsigned MIN / SUM mod 2^32 / OR --
the combination the reference's atomics produce in one pass, daq.cu:78-80)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn_name, out_dir):
    sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import torch.distributed as dist
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world)
    try:
        import test_shard
        res = getattr(test_shard, fn_name)(rank, world)
        np.save(os.path.join(out_dir, '%s_%d.npy' % (fn_name, rank)), res, allow_pickle=False)
    finally:
        dist.destroy_process_group()


def _run(fn_name, tmp_path, world=2):
    mp.spawn(_worker, args=(world, _free_port(), fn_name, str(tmp_path)), nprocs=world, join=True)
    return [np.load(os.path.join(str(tmp_path), '%s_%d.npy' % (fn_name, r))) for r in range(world)]


class _A(object):      # stands in for a GPUArray: a .tensor attribute
    def __init__(self, t):
        self.tensor = t


def _local_hits(rank):
    """rank r 'detects' 3 + 2r photons with recognisable words"""
    k = 3 + 2 * rank
    g = np.random.default_rng(rank)
    f = {n: _A(torch.from_numpy(g.random(k * w).astype(np.float32))) for n, w in
         (('pos', 3), ('dir', 3), ('pol', 3), ('wavelengths', 1), ('t', 1), ('weights', 1))}
    f['last_hit_triangles'] = _A(torch.arange(k, dtype=torch.int32) + 1000 * rank)
    f['flags'] = _A(torch.full((k,), 4 | (1 << 31), dtype=torch.int64).to(torch.int32))
    f['evidx'] = _A(torch.full((k,), rank, dtype=torch.int32))
    return f, _A(torch.arange(k, dtype=torch.int32) * 7 + rank)


def gather_hits(rank, world):
    from chroma.gpu import shard
    f, ch = _local_hits(rank)
    rows = shard.allgather_rows(shard.pack_hits(f, ch))
    hits = shard.unpack_hits(rows)
    return np.concatenate([hits.pos.ravel().view(np.uint32), hits.last_hit_triangles.view(np.uint32), hits.flags,
                           hits.evidx, hits.channel.view(np.uint32), hits.weights.view(np.uint32)])


def test_gather_hits_rank_order(tmp_path):
    from chroma.gpu import shard
    outs = _run('gather_hits', tmp_path)
    assert np.array_equal(outs[0], outs[1])          # every rank holds the same gathered hits
    exp = []
    for r in range(2):
        f, ch = _local_hits(r)
        exp.append(shard.unpack_hits(shard.pack_hits(f, ch)))
    pos = np.concatenate([e.pos for e in exp])
    want = np.concatenate([pos.ravel().view(np.uint32),
                           np.concatenate([e.last_hit_triangles for e in exp]).view(np.uint32),
                           np.concatenate([e.flags for e in exp]), np.concatenate([e.evidx for e in exp]),
                           np.concatenate([e.channel for e in exp]).view(np.uint32),
                           np.concatenate([e.weights for e in exp]).view(np.uint32)])
    assert np.array_equal(outs[0], want)
    assert np.concatenate([e.flags for e in exp])[0] == np.uint32(4 | (1 << 31))   # u32 bits survive


def empty_rank_gather(rank, world):
    from chroma.gpu import shard
    local = torch.arange(4 * rank, dtype=torch.int32).reshape(-1, 2) if rank else torch.zeros((0, 2), dtype=torch.int32)
    return shard.allgather_rows(local).numpy()


def gather_photons_end(rank, world):
    """keep_photons_end's gather (ShardedSimulation._photons_end): rank 1 holds
    5 end photons, rank 0 none; gathered to rank 0 in rank order."""
    from types import SimpleNamespace
    from chroma.gpu import shard
    f, _ = _local_hits(rank)
    if rank == 0:
        f = {k: _A(v.tensor[:0]) for k, v in f.items()}
    rows = shard.gather_rows(shard.pack_photons(SimpleNamespace(**f)), 0)
    if rows is None:
        return np.zeros(0, np.uint32)
    p = shard.unpack_photons(rows)
    return np.concatenate([p.pos.ravel().view(np.uint32), p.dir.ravel().view(np.uint32),
                           p.last_hit_triangles.view(np.uint32), p.flags, p.evidx, p.weights.view(np.uint32),
                           p.t.view(np.uint32)])


def test_gather_photons_end_to_root(tmp_path):
    from types import SimpleNamespace
    from chroma.gpu import shard
    outs = _run('gather_photons_end', tmp_path)
    assert outs[1].size == 0
    f, _ = _local_hits(1)
    p = shard.unpack_photons(shard.pack_photons(SimpleNamespace(**f)))
    assert len(p) == 5 and p.flags[0] == np.uint32(4 | (1 << 31)) and (p.evidx == 1).all()
    want = np.concatenate([p.pos.ravel().view(np.uint32), p.dir.ravel().view(np.uint32),
                           p.last_hit_triangles.view(np.uint32), p.flags, p.evidx, p.weights.view(np.uint32),
                           p.t.view(np.uint32)])
    assert np.array_equal(outs[0], want)
    assert np.array_equal(p.pos.ravel(), f['pos'].tensor.numpy()) and np.array_equal(p.t, f['t'].tensor.numpy())


def test_gather_with_an_empty_rank(tmp_path):
    outs = _run('empty_rank_gather', tmp_path)
    assert np.array_equal(outs[0], np.arange(4, dtype=np.int32).reshape(2, 2))
    assert np.array_equal(outs[1], outs[0])


def _daq_words(rank, n=37):
    g = np.random.default_rng(100 + rank)
    t = g.uniform(0, 50, n).astype(np.float32)
    t[g.random(n) < 0.3] = np.float32(1e9)            # channels this rank did not hit
    q = g.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)   # large: exercise the mod-2^32 wrap
    h = g.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    return t.view(np.uint32), q, h


def reduce_daq(rank, world):
    from chroma.gpu import shard
    t, q, h = (torch.from_numpy(x.view(np.int32).copy()) for x in _daq_words(rank))
    rt, rq, rh = shard.reduce_channels(t, q, h)
    c = shard.allreduce_channel_counts(torch.from_numpy(np.full(5, 2 ** 31 + rank, np.uint32).view(np.int32)))
    return np.concatenate([rt.numpy().view(np.uint32), rq.numpy().view(np.uint32), rh.numpy().view(np.uint32),
                           c.numpy().astype(np.uint64).astype(np.uint32), (c.numpy() >> 32).astype(np.uint32)])


def test_daq_channel_reduce(tmp_path):
    outs = _run('reduce_daq', tmp_path)
    assert np.array_equal(outs[0], outs[1])
    w = [_daq_words(r) for r in range(2)]
    t = np.minimum(w[0][0], w[1][0])                     # unsigned min of the time bits
    q = (w[0][1].astype(np.uint64) + w[1][1]).astype(np.uint32)
    h = w[0][2] | w[1][2]
    counts = np.full(5, (2 ** 31) * 2 + 1, np.uint64)    # int64 sum: no wrap for the counts
    want = np.concatenate([t, q, h, counts.astype(np.uint32), (counts >> 32).astype(np.uint32)])
    assert np.array_equal(outs[0], want)
    tf = t.view(np.float32)
    assert ((tf < 1e8) == ((w[0][0].view(np.float32) < 1e8) | (w[1][0].view(np.float32) < 1e8))).all()


def test_shard_range_partitions():
    from chroma.gpu.shard import shard_range
    for n in (0, 1, 7, 1000, 10_000_001):
        for world in (1, 2, 3, 8):
            r = [shard_range(n, k, world) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1


def seed_agreement(rank, world):
    from chroma.sim import agree_seed, pick_seed
    mine = pick_seed() + 7919 * rank          # ranks draw different seeds
    return np.array([mine, agree_seed(mine)], dtype=np.int64)


def test_seed_none_agrees_across_ranks(tmp_path):
    """ShardedSimulation(seed=None): rank 0's seed reaches every rank (the
    seed collective of the seed=None path)."""
    r0, r1 = _run('seed_agreement', tmp_path)
    assert r0[1] == r0[0] and r1[1] == r0[0] and r1[0] != r0[0]


def gather_root(rank, world):
    """hits to rank 0 only (ShardedSimulation(hits='root')): rank 1 gets None"""
    from chroma.gpu import shard
    f, ch = _local_hits(rank)
    rows = shard.gather_rows(shard.pack_hits(f, ch), dst=0)
    empty = shard.gather_rows(torch.zeros((0, 16), dtype=torch.int32), dst=0)
    if rank != 0:
        assert rows is None and empty is None
        return np.zeros(0, np.int32)
    assert empty.shape == (0, 16)
    return rows.numpy()


def test_gather_hits_to_root(tmp_path):
    from chroma.gpu import shard
    outs = _run('gather_root', tmp_path)
    want = torch.cat([shard.pack_hits(*_local_hits(r)) for r in range(2)]).numpy()
    assert np.array_equal(outs[0], want)
    assert outs[1].size == 0


def gather_root_world3(rank, world):
    from chroma.gpu import shard
    local = torch.full((rank, 3), rank, dtype=torch.int32)      # rank 0 contributes no rows
    rows = shard.gather_rows(local, dst=0)
    return rows.numpy() if rank == 0 else np.zeros(0, np.int32)


def test_gather_to_root_world3_ragged(tmp_path):
    outs = _run('gather_root_world3', tmp_path, world=3)
    assert np.array_equal(outs[0], np.array([[1, 1, 1], [2, 2, 2], [2, 2, 2]], np.int32))
