"""Simulation driver (drop-in for reference chroma/sim.py:22-282).

Batches events (never splitting one), uploads photons, propagates them on the
device with the reference's launch shape (nthreads_per_block=512,
max_blocks=1024 -> 524,288 RNG slots) and splits the detected hits back into
events.  Photon tracking, GPU-resident inputs and the per-event DAQ
(run_daq=True, chroma.gpu.daq) are supported as in the reference.
"""
import os
import time
from types import SimpleNamespace

import numpy as np

from chroma import event
from chroma import gpu
from chroma.gpu import gpuarray as ga
from chroma.itertoolset import peek


def pick_seed():
    """A seed from the current time and process id."""
    return int(time.time()) ^ (os.getpid() << 16) & 2 ** 32 - 1


def agree_seed(seed, group=None):
    """Rank 0's seed on every rank of `group` (a sharded job draws one seed).  The
    value travels as a tensor on the backend's device: the rank's own GPU for
    RCCL (bound by the caller before this collective), the CPU for gloo."""
    import torch
    import torch.distributed as dist
    from chroma.gpu import shard
    if shard.dist_info(group)[1] <= 1:
        return seed
    on_gpu = torch.cuda.is_available() and dist.get_backend(group) != 'gloo'
    box = torch.tensor([seed], dtype=torch.int64,
                       device=torch.device('cuda', shard.local_device()) if on_gpu else 'cpu')
    dist.broadcast(box, src=0, group=group)
    return int(box.item())


class Simulation(object):
    def __init__(self, detector, seed=None, cuda_device=None, photon_tracking=False, nthreads_per_block=512,
                 max_blocks=1024):
        self.detector = detector
        self.nthreads_per_block = nthreads_per_block
        self.max_blocks = max_blocks
        self.photon_tracking = photon_tracking
        self.seed = pick_seed() if seed is None else seed
        np.random.seed(self.seed & 0xFFFFFFFF)
        self.context = gpu.create_cuda_context(cuda_device)
        if hasattr(detector, 'num_channels'):
            self.gpu_geometry = gpu.GPUDetector(detector)
            self.gpu_daq = gpu.GPUDaq(self.gpu_geometry) if self.gpu_geometry.nchannels > 0 else None
            self.gpu_pdf = gpu.GPUPDF()                # sim.py:45-46
            self.gpu_pdf_kernel = gpu.GPUKernelPDF()
        else:
            self.gpu_geometry = gpu.GPUGeometry(detector)
        self.rng_states = gpu.get_rng_states(self.nthreads_per_block * self.max_blocks, seed=self.seed)
        self.pdf_config = None

    def _simulate_batch(self, batch_events, keep_photons_beg=False, keep_photons_end=False, keep_hits=True,
                        keep_flat_hits=True, run_daq=False, max_steps=100, verbose=False):
        t0 = time.time()
        sources = [ev.photons_beg for ev in batch_events]
        bounds = np.cumsum(np.concatenate([[0], [len(s) for s in sources]]))
        src = self._stack_gpu_photon_sources(sources)
        if src is None:
            src = event.Photons.join(sources)
        gpu_photons = gpu.GPUPhotons(src, copy_flags=True, copy_triangles=False, copy_weights=False)
        tracking = gpu_photons.propagate(self.gpu_geometry, self.rng_states, nthreads_per_block=self.nthreads_per_block,
                                         max_blocks=self.max_blocks, max_steps=max_steps, track=self.photon_tracking)
        if verbose:
            print('Batch took %0.2f s' % (time.time() - t0))
        if keep_photons_end:
            photons_end = gpu_photons.get()
        has_channels = hasattr(self.detector, 'num_channels')
        if has_channels and (keep_hits or keep_flat_hits):
            batch_hits = gpu_photons.get_flat_hits(self.gpu_geometry)
        for i, (ev, (start, end)) in enumerate(zip(batch_events, zip(bounds[:-1], bounds[1:]))):
            if not keep_photons_beg:
                ev.photons_beg = None
            if self.photon_tracking:
                step_ids, step_photons = tracking
                tracks = [[] for _ in range(end - start)]
                for ids, photons in zip(step_ids, step_photons):
                    mask = (ids >= start) & (ids < end)
                    if not mask.any():
                        break
                    sel = photons[mask]
                    for k, pid in enumerate(ids[mask] - start):
                        tracks[pid].append(sel[k])
                ev.photon_tracks = [event.Photons.join(t, concatenate=False) if t else event.Photons()
                                    for t in tracks]
            if keep_photons_end:
                ev.photons_end = photons_end[start:end]
            if has_channels and (keep_hits or keep_flat_hits):
                ev_hits = batch_hits[batch_hits.evidx == i]
                if keep_hits:
                    ev.hits = {int(ch): ev_hits[ev_hits.channel == ch] for ch in np.unique(ev_hits.channel)}
                if keep_flat_hits:
                    ev.flat_hits = ev_hits
            if run_daq and getattr(self, 'gpu_daq', None) is not None:
                # per event, as the reference does (sim.py:143-152)
                self.gpu_daq.begin_acquire()
                self.gpu_daq.acquire(gpu_photons, self.rng_states, start_photon=int(start), nphotons=int(end - start),
                                     nthreads_per_block=self.nthreads_per_block, max_blocks=self.max_blocks)
                ev.channels = self.gpu_daq.end_acquire().get()
            yield ev

    @staticmethod
    def _is_gpu_photon_source(photons):
        return all(isinstance(getattr(photons, f, None), ga.GPUArray)
                   for f in ('pos', 'dir', 'pol', 'wavelengths', 't', 'evidx', 'flags'))

    @classmethod
    def _stack_gpu_photon_sources(cls, sources):
        """Join GPU-resident inputs on the device (sim.py:171-223)."""
        if not sources or not all(cls._is_gpu_photon_source(s) for s in sources):
            return None
        total = sum(len(s) for s in sources)
        fields = ('pos', 'dir', 'pol', 'wavelengths', 't', 'evidx', 'flags')
        out = {}
        for f in fields:
            dest = ga.empty(total, getattr(sources[0], f).dtype)
            off = 0
            for s in sources:
                n = len(s)
                if n:
                    dest[off:off + n].tensor.copy_(getattr(s, f)[:n].tensor)
                    off += n
            out[f] = dest
        out['true_nphotons'] = total
        return SimpleNamespace(**out)

    def simulate(self, iterable, keep_photons_beg=False, keep_photons_end=False, keep_hits=True,
                 keep_flat_hits=True, run_daq=False, max_steps=1000, photons_per_batch=1000000):
        if isinstance(iterable, event.Photons):
            first, iterable = iterable, [iterable]
        else:
            first, iterable = peek(iterable)
        if isinstance(first, event.Photons):
            iterable = (event.Event(photons_beg=x) for x in iterable)
        elif isinstance(first, event.Vertex):
            raise NotImplementedError('Vertex input not supported in Chroma')
        nphotons = 0
        batch = []
        kw = dict(keep_photons_beg=keep_photons_beg, keep_photons_end=keep_photons_end, keep_hits=keep_hits,
                  keep_flat_hits=keep_flat_hits, run_daq=run_daq, max_steps=max_steps)
        for ev in iterable:
            ev.nphotons = len(ev.photons_beg)
            idx = len(batch)
            evidx = getattr(ev.photons_beg, 'evidx', None)
            if evidx is not None:
                if isinstance(evidx, ga.GPUArray):
                    if ev.nphotons > 0:
                        evidx[:ev.nphotons].fill(np.uint32(idx))
                else:
                    evidx[:ev.nphotons] = np.uint32(idx)
            nphotons += ev.nphotons
            batch.append(ev)
            if nphotons >= photons_per_batch:
                yield from self._simulate_batch(batch, **kw)
                nphotons, batch = 0, []
        if batch:
            yield from self._simulate_batch(batch, **kw)

    def __del__(self):
        ctx = getattr(self, 'context', None)
        if ctx is not None:
            try:
                ctx.pop()
            except Exception:
                pass


class ShardedSimulation(Simulation):
    """Simulation across the ranks of a torch.distributed job, one process per
    GPU (launch with torchrun; backend "nccl" = RCCL).  Every rank must call
    simulate() with the same events; each propagates its contiguous share of
    every batch on its own GPU (geometry replicated), then the detected hits
    are gathered in global photon order and the per-event DAQ channels are
    reduced (chroma.gpu.shard).  Every rank yields the same, complete events,
    equal to a single-GPU run's except for the RNG streams of ranks > 0
    (rank r draws from curand subsequences r*S .. r*S+S-1).
    photon_tracking and keep_photons_end are not sharded (use Simulation)."""

    def __init__(self, detector, seed=None, group=None, nthreads_per_block=512, max_blocks=1024):
        import torch
        import torch.distributed as dist
        from chroma.gpu import shard
        self.group = group
        self.rank, self.world = shard.dist_info(group)
        # bind this rank's GPU before any collective: RCCL stages on the current
        # device, which is cuda:0 on every rank unless set (all ranks would collide)
        if torch.cuda.is_available():
            torch.cuda.set_device(shard.local_device())
        if seed is None:
            seed = agree_seed(pick_seed(), group)
        Simulation.__init__(self, detector, seed=seed, cuda_device=shard.local_device(),
                            nthreads_per_block=nthreads_per_block, max_blocks=max_blocks)
        nslots = self.nthreads_per_block * self.max_blocks
        if self.rank:
            self.rng_states = gpu.get_rng_states(nslots, seed=self.seed, first_subsequence=self.rank * nslots)
        self._torch = torch

    def _simulate_batch(self, batch_events, keep_photons_beg=False, keep_photons_end=False, keep_hits=True,
                        keep_flat_hits=True, run_daq=False, max_steps=100, verbose=False):
        from chroma.gpu import shard
        if keep_photons_end:
            raise NotImplementedError('ShardedSimulation: keep_photons_end is not gathered; use Simulation')
        torch = self._torch
        sources = [ev.photons_beg for ev in batch_events]
        bounds = np.cumsum(np.concatenate([[0], [len(s) for s in sources]])).astype(np.int64)
        total = int(bounds[-1])
        lo, hi = shard.shard_range(total, self.rank, self.world)
        src = self._stack_gpu_photon_sources(sources)
        if src is None:
            local = event.Photons.join(sources)[lo:hi]
        else:
            local = SimpleNamespace(**{f: getattr(src, f)[lo:hi] for f in
                                       ('pos', 'dir', 'pol', 'wavelengths', 't', 'evidx', 'flags')})
            local.true_nphotons = hi - lo
        gpu_photons = gpu.GPUPhotons(local, copy_flags=True, copy_triangles=False, copy_weights=False)
        if hi > lo:
            gpu_photons.propagate(self.gpu_geometry, self.rng_states, nthreads_per_block=self.nthreads_per_block,
                                  max_blocks=self.max_blocks, max_steps=max_steps)
        has_channels = hasattr(self.detector, 'num_channels')
        if has_channels and (keep_hits or keep_flat_hits):
            fields, channels = gpu_photons.flat_hits_device(self.gpu_geometry)
            batch_hits = shard.unpack_hits(shard.allgather_rows(shard.pack_hits(fields, channels), self.group))
        for i, (ev, (start, end)) in enumerate(zip(batch_events, zip(bounds[:-1], bounds[1:]))):
            if not keep_photons_beg:
                ev.photons_beg = None
            if has_channels and (keep_hits or keep_flat_hits):
                ev_hits = batch_hits[batch_hits.evidx == i]
                if keep_hits:
                    ev.hits = {int(ch): ev_hits[ev_hits.channel == ch] for ch in np.unique(ev_hits.channel)}
                if keep_flat_hits:
                    ev.flat_hits = ev_hits
            if run_daq and getattr(self, 'gpu_daq', None) is not None:
                daq = self.gpu_daq
                daq.begin_acquire()
                a, b = max(int(start), lo), min(int(end), hi)     # this rank's part of the event
                if b > a:
                    daq.acquire(gpu_photons, self.rng_states, start_photon=a - lo, nphotons=b - a,
                                nthreads_per_block=self.nthreads_per_block, max_blocks=self.max_blocks)
                t, q, h = shard.reduce_channels(daq.earliest_time_int_gpu.tensor, daq.channel_q_int_gpu.tensor,
                                                daq.channel_history_gpu.tensor, self.group)
                daq.earliest_time_int_gpu.tensor.copy_(t)
                daq.channel_q_int_gpu.tensor.copy_(q)
                daq.channel_history_gpu.tensor.copy_(h)
                ev.channels = daq.end_acquire().get()
            yield ev
