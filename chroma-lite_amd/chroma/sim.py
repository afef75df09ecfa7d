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


class _Batch(object):
    """One batch of events on the device: its GPUPhotons (uploaded when the
    batch closes, before a later batch can restamp a shared source's evidx),
    the event bounds in the batch's photon range, and this process's part of
    that range ([lo, hi): everything for Simulation, a shard for
    ShardedSimulation)."""
    __slots__ = ('events', 'gpu_photons', 'bounds', 'lo', 'hi', 'tracking')

    def __init__(self, events, gpu_photons, bounds, lo, hi):
        self.events, self.gpu_photons, self.bounds, self.lo, self.hi = events, gpu_photons, bounds, lo, hi
        self.tracking = None


class Simulation(object):
    # batches propagated per chr_propagate_batches call by simulate(): batch k's
    # multi-step tail (its longest-lived photon's serial chain) runs on a second
    # HIP stream under batch k+1's first step; results are bit-identical to one
    # propagate per batch (tests/test_gpu_sim_pipeline.py).  1 = the reference's
    # one-batch-at-a-time loop (sim.py:116-160).
    pipeline_batches = 8

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
        self.last_pipeline = None     # (batches, propagate_batches calls) of the last simulate()

    # ------------------------------------------------------------ batch stages
    def _upload(self, batch_events):
        """The batch's photons on the device (sim.py:54-70)."""
        sources = [ev.photons_beg for ev in batch_events]
        bounds = np.cumsum(np.concatenate([[0], [len(s) for s in sources]])).astype(np.int64)
        src = self._stack_gpu_photon_sources(sources)
        if src is None:
            src = event.Photons.join(sources)
        gpu_photons = gpu.GPUPhotons(src, copy_flags=True, copy_triangles=False, copy_weights=False)
        return _Batch(batch_events, gpu_photons, bounds, 0, int(bounds[-1]))

    def _propagate(self, batches, max_steps):
        """Propagate the batches in order with the one rng_states: one
        pipelined chr_propagate_batches call for several (chroma.gpu.propagate_batches),
        GPUPhotons.propagate for one or with photon tracking."""
        kw = dict(nthreads_per_block=self.nthreads_per_block, max_blocks=self.max_blocks, max_steps=max_steps)
        live = [b for b in batches if b.hi > b.lo]
        if len(live) > 1 and not self.photon_tracking:
            gpu.propagate_batches([b.gpu_photons for b in live], self.gpu_geometry, self.rng_states, **kw)
            return 1
        for b in live:
            b.tracking = b.gpu_photons.propagate(self.gpu_geometry, self.rng_states, track=self.photon_tracking, **kw)
        return 0

    def _batch_hits(self, b):
        return b.gpu_photons.get_flat_hits(self.gpu_geometry)

    def _photons_end(self, b):
        """The batch's photons after propagation, batch order (sim.py:72-75)."""
        return b.gpu_photons.get()

    def _acquire(self, b, start, end):
        """DAQ of one event (sim.py:143-152)."""
        self.gpu_daq.begin_acquire()
        self.gpu_daq.acquire(b.gpu_photons, self.rng_states, start_photon=int(start), nphotons=int(end - start),
                             nthreads_per_block=self.nthreads_per_block, max_blocks=self.max_blocks)
        return self.gpu_daq.end_acquire().get()

    def _emit(self, b, keep_photons_beg=False, keep_photons_end=False, keep_hits=True, keep_flat_hits=True,
              run_daq=False):
        """Split a propagated batch back into its events (sim.py:72-110)."""
        if keep_photons_end:
            photons_end = self._photons_end(b)
        has_channels = hasattr(self.detector, 'num_channels')
        batch_hits = None
        if has_channels and (keep_hits or keep_flat_hits):
            batch_hits = self._batch_hits(b)
        for i, (ev, (start, end)) in enumerate(zip(b.events, zip(b.bounds[:-1], b.bounds[1:]))):
            if not keep_photons_beg:
                ev.photons_beg = None
            if self.photon_tracking:
                step_ids, step_photons = b.tracking
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
                ev.photons_end = photons_end[start:end] if photons_end is not None else None
            if batch_hits is not None:
                ev_hits = batch_hits[batch_hits.evidx == i]
                if keep_hits:
                    ev.hits = {int(ch): ev_hits[ev_hits.channel == ch] for ch in np.unique(ev_hits.channel)}
                if keep_flat_hits:
                    ev.flat_hits = ev_hits
            if run_daq and getattr(self, 'gpu_daq', None) is not None:
                ev.channels = self._acquire(b, start, end)
            yield ev

    def _simulate_batch(self, batch_events, keep_photons_beg=False, keep_photons_end=False, keep_hits=True,
                        keep_flat_hits=True, run_daq=False, max_steps=100, verbose=False):
        """One batch, as the reference's _simulate_batch (sim.py:54-110)."""
        t0 = time.time()
        b = self._upload(batch_events)
        self._propagate([b], max_steps)
        if verbose:
            print('Batch took %0.2f s' % (time.time() - t0))
        yield from self._emit(b, keep_photons_beg=keep_photons_beg, keep_photons_end=keep_photons_end,
                              keep_hits=keep_hits, keep_flat_hits=keep_flat_hits, run_daq=run_daq)

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

    def _pipeline_depth(self, run_daq):
        """Batches per propagate call: 1 where the reference's interleaving is
        observable -- the DAQ draws from rng_states between two batches'
        propagates, photon tracking downloads every step."""
        if run_daq or self.photon_tracking:
            return 1
        return max(1, int(self.pipeline_batches))

    def simulate(self, iterable, keep_photons_beg=False, keep_photons_end=False, keep_hits=True,
                 keep_flat_hits=True, run_daq=False, max_steps=1000, photons_per_batch=1000000):
        """sim.py:112-160.  Events are batched as the reference batches them
        (never split, a batch closes once it holds photons_per_batch photons)
        and yielded in order; up to pipeline_batches closed batches are
        propagated in one pipelined call (read ahead from the iterable), with
        results bit-identical to the reference's one-batch-at-a-time loop."""
        if isinstance(iterable, event.Photons):
            first, iterable = iterable, [iterable]
        else:
            first, iterable = peek(iterable)
        if isinstance(first, event.Photons):
            iterable = (event.Event(photons_beg=x) for x in iterable)
        elif isinstance(first, event.Vertex):
            raise NotImplementedError('Vertex input not supported in Chroma')
        emit_kw = dict(keep_photons_beg=keep_photons_beg, keep_photons_end=keep_photons_end, keep_hits=keep_hits,
                       keep_flat_hits=keep_flat_hits, run_daq=run_daq)
        depth = self._pipeline_depth(run_daq)
        stats = [0, 0]
        pending = []

        def flush():
            stats[0] += len(pending)
            stats[1] += self._propagate(pending, max_steps)
            for b in pending:
                yield from self._emit(b, **emit_kw)
            del pending[:]

        nphotons = 0
        batch = []
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
                pending.append(self._upload(batch))
                nphotons, batch = 0, []
                if len(pending) >= depth:
                    yield from flush()
        if batch:
            pending.append(self._upload(batch))
        if pending:
            yield from flush()
        self.last_pipeline = tuple(stats)

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
    every batch on its own GPU (geometry replicated; a rank's batches are
    pipelined as Simulation's), then the detected hits are gathered in global
    photon order -- to rank 0 only (hits='root', the default: other ranks'
    events carry hits/flat_hits None) or to every rank (hits='all') -- and the
    per-event DAQ channels are reduced on every rank (chroma.gpu.shard).  The
    events equal a single-GPU run's except for the RNG streams of ranks > 0
    (rank r draws from curand subsequences r*S .. r*S+S-1).  keep_photons_end
    gathers the end photons the same way as the hits (to rank 0, or to every
    rank with hits='all'; None elsewhere).  photon_tracking is not sharded (use
    Simulation)."""

    def __init__(self, detector, seed=None, group=None, nthreads_per_block=512, max_blocks=1024, hits='root'):
        import torch
        from chroma.gpu import shard
        if hits not in ('root', 'all'):
            raise ValueError("hits must be 'root' or 'all'")
        self.hits_to = hits
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

    def _upload(self, batch_events):
        from chroma.gpu import shard
        sources = [ev.photons_beg for ev in batch_events]
        bounds = np.cumsum(np.concatenate([[0], [len(s) for s in sources]])).astype(np.int64)
        lo, hi = shard.shard_range(int(bounds[-1]), self.rank, self.world)
        src = self._stack_gpu_photon_sources(sources)
        if src is None:
            local = event.Photons.join(sources)[lo:hi]
        else:
            local = SimpleNamespace(**{f: getattr(src, f)[lo:hi] for f in
                                       ('pos', 'dir', 'pol', 'wavelengths', 't', 'evidx', 'flags')})
            local.true_nphotons = hi - lo
        gpu_photons = gpu.GPUPhotons(local, copy_flags=True, copy_triangles=False, copy_weights=False)
        return _Batch(batch_events, gpu_photons, bounds, lo, hi)

    def _batch_hits(self, b):
        from chroma.gpu import shard
        fields, channels = b.gpu_photons.flat_hits_device(self.gpu_geometry)
        rows = shard.pack_hits(fields, channels)
        if self.hits_to == 'all':
            return shard.unpack_hits(shard.allgather_rows(rows, self.group))
        rows = shard.gather_rows(rows, 0, self.group)
        return shard.unpack_hits(rows) if rows is not None else None

    def _photons_end(self, b):
        """Every rank's shard of the batch's end photons, concatenated in rank
        (= global photon) order on rank 0 (hits='root'; None on the others) or on
        every rank (hits='all')."""
        from chroma.gpu import shard
        rows = shard.pack_photons(b.gpu_photons)
        if self.hits_to == 'all':
            return shard.unpack_photons(shard.allgather_rows(rows, self.group))
        rows = shard.gather_rows(rows, 0, self.group)
        return shard.unpack_photons(rows) if rows is not None else None

    def _acquire(self, b, start, end):
        from chroma.gpu import shard
        daq = self.gpu_daq
        daq.begin_acquire()
        a, c = max(int(start), b.lo), min(int(end), b.hi)     # this rank's part of the event
        if c > a:
            daq.acquire(b.gpu_photons, self.rng_states, start_photon=a - b.lo, nphotons=c - a,
                        nthreads_per_block=self.nthreads_per_block, max_blocks=self.max_blocks)
        t, q, h = shard.reduce_channels(daq.earliest_time_int_gpu.tensor, daq.channel_q_int_gpu.tensor,
                                        daq.channel_history_gpu.tensor, self.group)
        daq.earliest_time_int_gpu.tensor.copy_(t)
        daq.channel_q_int_gpu.tensor.copy_(q)
        daq.channel_history_gpu.tensor.copy_(h)
        return daq.end_acquire().get()
