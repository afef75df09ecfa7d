"""Photon-sharded multi-GPU runs: one process per GPU, torch.distributed
(backend "nccl", which is RCCL over xGMI on ROCm).

Photons are independent and the geometry is read-only, so the path shards
without any exchange during propagation: every rank
holds a full replica of the geometry in its own HBM and propagates a
contiguous slice of each batch.  Collectives appear only where the reference
path has a reduction step:

  * detected hits (GPUPhotons.get_flat_hits, reference photon.py:141-209) are
    gathered in rank order, which is ascending global photon order -- the same
    order a single-GPU run returns -- to rank 0 (gather_rows), or to every
    rank when each needs the events (allgather_rows);
  * the DAQ's per-channel words (reference daq.cu:78-80: atomicMin of the time
    bits, atomicAdd of the quantised charge, atomicOr of the history) are
    reduced with the same three operators: unsigned MIN, SUM (mod 2^32, as the
    u32 atomics wrap) and OR (RCCL has no bitwise reduction: the per-rank words
    are all-gathered -- 8 x 116 KB for 29k channels -- and OR-ed on device);
  * per-channel hit counts (chr_channel_hit_counts) are SUM-reduced;
  * the end photons (keep_photons_end) are gathered like the hits, in global
    photon order (pack_photons).

RNG streams: rank r of a world of W initialises its S slot states as
curand_init(seed, r*S + slot) (get_rng_states(first_subsequence=r*S)), so no
two ranks share a stream and rank 0 of any world draws exactly what a
single-GPU run draws.

The collective helpers work on any torch.distributed backend (gloo on CPU
tensors for the host tests, RCCL on device tensors in production).
"""
import os

import numpy as np
import torch

from chroma import event

# one gathered hit record: pos(3) dir(3) pol(3) wavelength t weight (f32 bits),
# last_hit flags evidx channel (i32/u32 bits) -> 16 words = 64 bytes
HIT_WORDS = 16


def dist_info(group=None):
    """(rank, world size) of the default (or given) process group; (0, 1) when
    torch.distributed is not initialised."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def shard_range(n, rank, world):
    """Contiguous slice [lo, hi) of n photons owned by `rank`."""
    return n * rank // world, n * (rank + 1) // world


def _host_backend(group):
    """gloo (host tests, or ranks sharing one GPU) moves device tensors through
    host memory; RCCL works on them in place."""
    import torch.distributed as dist
    return dist.get_backend(group) == 'gloo'


def _all_gather(parts, t, group):
    import torch.distributed as dist
    if t.is_cuda and _host_backend(group):
        host = [torch.empty_like(t, device='cpu') for _ in parts]
        dist.all_gather(host, t.cpu(), group=group)
        for p, h in zip(parts, host):
            p.copy_(h)
    else:
        dist.all_gather(parts, t, group=group)


def _gather(parts, t, dst, group):
    """dist.gather of t into parts (on dst; parts is None elsewhere)."""
    import torch.distributed as dist
    if t.is_cuda and _host_backend(group):
        host = [torch.empty_like(t, device='cpu') for _ in parts] if parts is not None else None
        dist.gather(t.cpu(), host, dst=dst, group=group)
        if parts is not None:
            for p, h in zip(parts, host):
                p.copy_(h)
    else:
        dist.gather(t, parts, dst=dst, group=group)


def _all_reduce(t, op, group):
    import torch.distributed as dist
    if t.is_cuda and _host_backend(group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


def allgather_rows(local, group=None):
    """All-gather a (k_r, W) tensor from every rank; returns the (sum k_r, W)
    concatenation in rank order (rows are padded to max k_r for the collective)."""
    import torch.distributed as dist
    rank, world = dist_info(group)
    if world == 1:
        return local
    k = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    ks = [torch.zeros_like(k) for _ in range(world)]
    _all_gather(ks, k, group)
    counts = [int(x.item()) for x in ks]
    m = max(counts)
    if m == 0:
        return local[:0]
    padded = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    padded[:local.shape[0]] = local
    parts = [torch.empty_like(padded) for _ in range(world)]
    _all_gather(parts, padded, group)
    return torch.cat([parts[r][:counts[r]] for r in range(world)])


def gather_rows(local, dst=0, group=None):
    """Gather a (k_r, W) tensor from every rank to rank `dst` only: returns the
    (sum k_r, W) concatenation in rank order on dst, None on the other ranks.
    Only the row counts travel to every rank (W*8 bytes); the rows themselves
    cross xGMI once, to dst (rows padded to max k_r for the collective)."""
    import torch.distributed as dist
    rank, world = dist_info(group)
    if world == 1:
        return local
    k = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    ks = [torch.zeros_like(k) for _ in range(world)]
    _all_gather(ks, k, group)
    counts = [int(x.item()) for x in ks]
    m = max(counts)
    root = dist.get_global_rank(group, dst) if group is not None else dst
    if m == 0:
        return local[:0] if rank == dst else None
    padded = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    padded[:local.shape[0]] = local
    parts = [torch.empty_like(padded) for _ in range(world)] if rank == dst else None
    _gather(parts, padded, root, group)
    if rank != dst:
        return None
    return torch.cat([parts[r][:counts[r]] for r in range(world)])


def _u32_to_i64(t):
    return t.to(torch.int64) & 0xFFFFFFFF


def _i64_to_u32bits(t):
    t = t & 0xFFFFFFFF
    return torch.where(t >= 2 ** 31, t - 2 ** 32, t).to(torch.int32)


def allreduce_channel_counts(counts, group=None):
    """SUM of per-channel u32 counts (stored as int32 bits) over ranks; returns int64."""
    import torch.distributed as dist
    c = _u32_to_i64(counts)
    if dist_info(group)[1] > 1:
        _all_reduce(c, dist.ReduceOp.SUM, group)
    return c


def reduce_channels(time_int, q_int, history, group=None):
    """Combine the per-rank DAQ words (int32 tensors holding u32 bits, as
    GPUDaq keeps them) exactly as the reference's atomics would have combined
    them in one DAQ pass: time = unsigned min, q = sum mod 2^32, history = OR.
    Returns three int32 tensors (u32 bits)."""
    import torch.distributed as dist
    rank, world = dist_info(group)
    if world == 1:
        return time_int, q_int, history
    t = _u32_to_i64(time_int)
    _all_reduce(t, dist.ReduceOp.MIN, group)
    q = _u32_to_i64(q_int)
    _all_reduce(q, dist.ReduceOp.SUM, group)
    parts = [torch.empty_like(history) for _ in range(world)]
    _all_gather(parts, history.contiguous(), group)
    h = parts[0].clone()
    for p in parts[1:]:
        h |= p
    return _i64_to_u32bits(t), _i64_to_u32bits(q), h


def pack_hits(fields, channels):
    """(k, 16) int32 tensor of hit records from device photon arrays (dict of
    GPUArrays as GPUPhotons.flat_hits_device returns) and the channel array."""
    k = channels.tensor.numel()
    if k == 0:
        return torch.zeros((0, HIT_WORDS), dtype=torch.int32, device=channels.tensor.device)

    def f32(a, w):
        return a.tensor.view(torch.int32).reshape(k, w)

    def i32(a):
        return a.tensor.reshape(k, 1)
    return torch.cat([f32(fields['pos'], 3), f32(fields['dir'], 3), f32(fields['pol'], 3),
                      f32(fields['wavelengths'], 1), f32(fields['t'], 1), f32(fields['weights'], 1),
                      i32(fields['last_hit_triangles']), i32(fields['flags']), i32(fields['evidx']),
                      i32(channels)], dim=1)


# one gathered photon (keep_photons_end): the hit record without the channel -> 15 words
PHOTON_WORDS = 15


def pack_photons(gp):
    """(n, 15) int32 tensor of every photon of a GPUPhotons (or any object with
    the nine photon GPUArrays), in photon order: the end photons a sharded run
    gathers for keep_photons_end (reference sim.py:72-75 downloads them whole)."""
    k = gp.wavelengths.tensor.numel()
    if k == 0:
        return torch.zeros((0, PHOTON_WORDS), dtype=torch.int32, device=gp.wavelengths.tensor.device)

    def f32(a, w):
        return a.tensor.view(torch.int32).reshape(k, w)

    def i32(a):
        return a.tensor.view(torch.int32).reshape(k, 1)
    return torch.cat([f32(gp.pos, 3), f32(gp.dir, 3), f32(gp.pol, 3), f32(gp.wavelengths, 1), f32(gp.t, 1),
                      f32(gp.weights, 1), i32(gp.last_hit_triangles), i32(gp.flags), i32(gp.evidx)], dim=1)


def unpack_photons(rows):
    """event.Photons from gathered (K, 15) photon records."""
    a = rows.cpu().numpy()
    f = a.view(np.float32)
    return event.Photons(f[:, 0:3].copy(), f[:, 3:6].copy(), f[:, 6:9].copy(), f[:, 9].copy(), f[:, 10].copy(),
                         a[:, 12].copy(), a[:, 13].view(np.uint32).copy(), f[:, 11].copy(),
                         a[:, 14].view(np.uint32).copy())


def unpack_hits(rows):
    """event.Photons (with .channel) from gathered (K, 16) hit records."""
    a = rows.cpu().numpy()
    f = a.view(np.float32)
    return event.Photons(f[:, 0:3].copy(), f[:, 3:6].copy(), f[:, 6:9].copy(), f[:, 9].copy(), f[:, 10].copy(),
                         a[:, 12].copy(), a[:, 13].view(np.uint32).copy(), f[:, 11].copy(),
                         a[:, 14].view(np.uint32).copy(), a[:, 15].copy())


def local_device():
    """The GPU this rank drives: LOCAL_RANK (torchrun) or 0."""
    return int(os.environ.get('LOCAL_RANK', '0'))
