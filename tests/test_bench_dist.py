"""bench.py's multi-rank scaffolding on CPU (gloo, world size 2), the code the
driver's N>1 bench runs around the propagate step: rank 0 builds the geometry
and fills the node-local cache while the other ranks wait at a barrier and
then load it; per-rank RNG subsequences are disjoint; the timed loop brackets
its steps with barriers and reports the MAX over ranks; each step SUM-reduces
the per-channel hit counts (chroma.gpu.shard.allreduce_channel_counts).  The
propagate itself needs a GPU and is covered by the -m gpu tests."""
import os
import socket
import sys
import time

import numpy as np
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d' % port, rank=rank, world_size=world)
    try:
        import bench
        from chroma.gpu import shard
        cache = os.path.join(out_dir, 'cache')
        det = bench.shared_geometry('small', cache, rank, dist)
        md5 = int(det.mesh.md5()[:12], 16)
        nch = det.num_channels()
        counts = torch.zeros(nch, dtype=torch.int32)
        reduced = {}

        def run(m):   # m steps per call, as bench.py's pipelined groups
            out = []
            for _ in range(m):
                time.sleep(0.02 * (rank + 1))               # rank 1 is the slow one
                counts.fill_(0)
                counts[rank % nch] = 3 + rank                # this rank's "hits"
                reduced['c'] = shard.allreduce_channel_counts(counts)
                out.append(rank)
            return out

        elapsed, per_step, results = bench.timed_loop(run, 3, 1, dist, lambda: None, group=2)
        c = reduced['c'].numpy()
        res = np.array([elapsed, sum(per_step), md5, nch, bench.rng_first_subsequence(rank, 524288),
                        c[0], c[1 % nch], c.sum(), len(results)], dtype=np.float64)
        np.save(os.path.join(out_dir, 'r%d.npy' % rank), res, allow_pickle=False)
    finally:
        dist.destroy_process_group()


def test_bench_world2_scaffolding(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (np.load(os.path.join(str(tmp_path), 'r%d.npy' % r)) for r in range(2))
    # one geometry, built once by rank 0 into the shared cache, loaded by rank 1
    assert r0[2] == r1[2] and r0[3] == r1[3]
    assert os.path.isdir(os.path.join(str(tmp_path), 'cache'))
    # timed region: max over ranks -> identical on both, at least the slow rank's 3 steps
    assert r0[0] == r1[0] and r0[0] >= 3 * 0.04 - 1e-3
    assert r1[1] >= 3 * 0.04 - 1e-3
    # disjoint RNG subsequences: rank r starts at r * nslots
    assert (r0[4], r1[4]) == (0, 524288)
    # the per-step channel reduce: rank 0 put 3 in channel 0, rank 1 put 4 in channel 1
    for r in (r0, r1):
        assert r[5] == 3 and r[6] == 4 and r[7] == 7 and r[8] == 3
