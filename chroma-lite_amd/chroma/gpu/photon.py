"""GPUPhotons (drop-in for reference chroma/gpu/photon.py:13-415).

Same constructor, attributes (pos dir pol wavelengths t last_hit_triangles
flags weights evidx true_nphotons ncopies) and methods; device work goes
through the C ABI (libchroma_amd.so): chr_propagate for the whole host step
loop of photon.py:226-293, chr_propagate_chunk when tracking, chr_photon_hits
(count_photon_hits/copy_photon_hits), chr_select_photons (count_photons/
copy_photons), chr_copy_photon_queue and chr_photon_duplicate.

Differences from the reference, all deliberate:
 * survivors are enqueued in input order (stable compaction), so a propagate
   is deterministic for a given seed; the reference's warp-atomic order is
   not;
 * hit/selection outputs are in ascending photon order;
 * evidx is allocated for all copies (the reference allocates nphotons and
   photon_duplicate writes nphotons*ncopies of it, photon.py:62 vs
   propagate.cu:66).
"""
import ctypes
import sys

import numpy as np

from chroma import event
from chroma.gpu import _native
from chroma.gpu import gpuarray as ga
from chroma.gpu.tools import chunk_iterator, current_stream, to_float3

_FIELDS = ('pos', 'dir', 'pol', 'wavelengths', 't', 'flags', 'last_hit_triangles', 'weights', 'evidx')


def _photons_desc(holder):
    return _native.PhotonsDesc(holder.pos.gpudata, holder.dir.gpudata, holder.pol.gpudata,
                               holder.wavelengths.gpudata, holder.t.gpudata, holder.weights.gpudata,
                               holder.flags.gpudata, holder.last_hit_triangles.gpudata, holder.evidx.gpudata)


def _alloc(n):
    return dict(pos=ga.empty(n, ga.vec.float3), dir=ga.empty(n, ga.vec.float3), pol=ga.empty(n, ga.vec.float3),
                wavelengths=ga.empty(n, np.float32), t=ga.empty(n, np.float32),
                last_hit_triangles=ga.empty(n, np.int32), flags=ga.empty(n, np.uint32),
                weights=ga.empty(n, np.float32), evidx=ga.empty(n, np.uint32))


def _resolve_nphotons(ph):
    try:
        return len(ph)
    except TypeError:
        pass
    n = getattr(ph, 'true_nphotons', None)
    if n is not None:
        return int(n)
    pos = getattr(ph, 'pos', None)
    if pos is not None:
        return len(pos)
    raise TypeError('Cannot determine photon count from object of type %r' % type(ph))


class GPUPhotons(object):
    def __init__(self, photons, ncopies=1, copy_flags=True, copy_triangles=True, copy_weights=True):
        nphotons = _resolve_nphotons(photons)
        total = nphotons * ncopies
        for k, v in _alloc(total).items():
            setattr(self, k, v)
        if not copy_triangles:
            self.last_hit_triangles.fill(-1)
        if not copy_flags:
            self.flags.fill(0)
        if not copy_weights:
            self.weights.fill(1.0)

        def copy_field(dest, source, dtype):
            head = dest[:nphotons]
            if isinstance(source, ga.GPUArray):
                count = min(len(source), nphotons)
                head.tensor[:source[:count].tensor.numel()].copy_(source[:count].tensor)
            elif dest.dtype == ga.vec.float3:
                head.set(to_float3(np.asarray(source, dtype=np.float32).reshape(-1, 3)))
            else:
                head.set(np.asarray(source, dtype=dtype))

        copy_field(self.pos, photons.pos, np.float32)
        copy_field(self.dir, photons.dir, np.float32)
        copy_field(self.pol, photons.pol, np.float32)
        copy_field(self.wavelengths, photons.wavelengths, np.float32)
        copy_field(self.t, photons.t, np.float32)
        if copy_triangles:
            copy_field(self.last_hit_triangles, photons.last_hit_triangles, np.int32)
        if copy_flags:
            copy_field(self.flags, photons.flags, np.uint32)
        if copy_weights:
            copy_field(self.weights, photons.weights, np.float32)
        copy_field(self.evidx, photons.evidx, np.uint32)
        if ncopies > 1:
            desc = _photons_desc(self)
            for first, count, _ in chunk_iterator(nphotons, 256, 1024):
                _native.call('chr_photon_duplicate', ctypes.byref(desc), first, count, ncopies - 1, nphotons,
                             current_stream())
        self.true_nphotons = getattr(photons, 'true_nphotons', nphotons)
        self.ncopies = ncopies

    # ---------------------------------------------------------------- host I/O
    def get(self):
        def vec3(a):
            return a.get().view(np.float32).reshape((len(a), 3))
        return event.Photons(vec3(self.pos), vec3(self.dir), vec3(self.pol), self.wavelengths.get(), self.t.get(),
                             self.last_hit_triangles.get(), self.flags.get(), self.weights.get(), self.evidx.get())

    def __len__(self):
        return self.pos.size

    def _desc(self):
        return _photons_desc(self)

    # ---------------------------------------------------------------- hits
    def get_hits(self, *args, **kwargs):
        flat = self.get_flat_hits(*args, **kwargs)
        return {int(ch): flat[flat.channel == ch] for ch in np.unique(flat.channel)}

    def flat_hits_device(self, gpu_detector, target_flag=(0x1 << 2), start_photon=None, nphotons=None):
        """Device-resident compacted hits: (dict of the nine photon GPUArrays,
        channel GPUArray i32), ascending photon order.  get_flat_hits() is this
        plus the download; the photon-sharded path gathers these over RCCL."""
        start = 0 if start_photon is None else start_photon
        n = self.pos.size - start if nphotons is None else nphotons
        desc = self._desc()
        count = ctypes.c_uint32()
        _native.call('chr_photon_hits', ctypes.byref(desc), start, n, int(target_flag),
                     gpu_detector.solid_id_map.gpudata, gpu_detector.solid_id_to_channel_index_gpu.gpudata,
                     None, None, ctypes.byref(count), current_stream())
        k = count.value
        out = _alloc(k)
        channels = ga.empty(k, np.int32)
        if k > 0:
            holder = type('H', (), out)()
            odesc = _photons_desc(holder)
            _native.call('chr_photon_hits', ctypes.byref(desc), start, n, int(target_flag),
                         gpu_detector.solid_id_map.gpudata, gpu_detector.solid_id_to_channel_index_gpu.gpudata,
                         ctypes.byref(odesc), channels.gpudata, ctypes.byref(count), current_stream())
            assert count.value == k
        return out, channels

    def get_flat_hits(self, gpu_detector, target_flag=(0x1 << 2), nthreads_per_block=256, max_blocks=1024,
                      start_photon=None, nphotons=None, no_map=False):
        """Detected photons: flags & target_flag, last_hit_triangle > -1 and
        a channel behind the hit solid; returns event.Photons with .channel."""
        out, channels = self.flat_hits_device(gpu_detector, target_flag, start_photon, nphotons)

        def vec3(a):
            return a.get().view(np.float32).reshape((len(a), 3))
        return event.Photons(vec3(out['pos']), vec3(out['dir']), vec3(out['pol']), out['wavelengths'].get(),
                             out['t'].get(), out['last_hit_triangles'].get(), out['flags'].get(),
                             out['weights'].get(), out['evidx'].get(), channels.get())

    def iterate_copies(self):
        for i in range(self.ncopies):
            w = slice(self.true_nphotons * i, self.true_nphotons * (i + 1))
            yield GPUPhotonsSlice(*[getattr(self, f)[w] for f in ('pos', 'dir', 'pol', 'wavelengths', 't',
                                                                  'last_hit_triangles', 'flags', 'weights',
                                                                  'evidx')])

    # ---------------------------------------------------------------- propagate
    def propagate(self, gpu_geometry, rng_states, nthreads_per_block=256, max_blocks=1024, max_steps=10,
                  use_weights=False, scatter_first=0, track=False):
        """Propagate to termination or max_steps (photon.py:226-293).

        rng_states must hold at least nthreads_per_block*max_blocks states.
        Returns (step_photon_ids, step_photons) when track=True.
        """
        nphotons = self.pos.size
        nslots = len(rng_states)
        if nthreads_per_block * max_blocks > nslots:
            raise ValueError('rng_states must have at least nthreads_per_block*max_blocks states')
        if not track:
            stats = _native.PropagateStats()
            _native.call('chr_propagate', ctypes.c_void_p(gpu_geometry.gpudata), ctypes.byref(self._desc()),
                         nphotons, self.true_nphotons, self.ncopies, rng_states.gpudata, nslots,
                         nthreads_per_block, max_blocks, max_steps, int(bool(use_weights)), int(scatter_first),
                         ctypes.byref(stats), current_stream())
            self.last_stats = stats
            if stats.stack_overflows:
                print('WARNING: %d BVH traversals exceeded the 1000-entry stack' % stats.stack_overflows,
                      file=sys.stderr)
            return None
        return self._propagate_tracked(gpu_geometry, rng_states, nthreads_per_block, max_blocks, max_steps,
                                       use_weights, scatter_first)

    def _propagate_tracked(self, gpu_geometry, rng_states, ntpb, max_blocks, max_steps, use_weights,
                           scatter_first):
        nphotons = self.pos.size
        queue = np.empty(nphotons + 1, dtype=np.uint32)
        queue[0] = 0
        for c in range(self.ncopies):
            queue[1 + c::self.ncopies] = np.arange(self.true_nphotons, dtype=np.uint32) + c * self.true_nphotons
        qin = ga.to_gpu(queue)
        out = np.zeros(nphotons + 1, dtype=np.uint32)
        out[0] = 1
        qout = ga.to_gpu(out)
        scratch = ga.empty(int(_native.lib().chr_propagate_scratch_words(min(nphotons, ntpb * max_blocks))),
                           np.uint32)
        scratch.fill(0)
        desc = self._desc()
        step_photon_ids = [qin[1:nphotons + 1].get()]
        step_photons = [self.copy_queue(qin[1:], nphotons).get()]
        step = 0
        while step < max_steps:
            for first, count, _ in chunk_iterator(nphotons, ntpb, max_blocks):
                _native.call('chr_propagate_chunk', ctypes.c_void_p(gpu_geometry.gpudata), ctypes.byref(desc),
                             rng_states.gpudata, len(rng_states), first, count, qin[1:].gpudata, qout.gpudata, 1,
                             int(bool(use_weights)), int(scatter_first), scratch.gpudata, current_stream())
            step_photon_ids.append(qin[1:nphotons + 1].get())
            step_photons.append(self.copy_queue(qin[1:], nphotons).get())
            step += 1
            scatter_first = 0
            if step < max_steps:
                qin, qout = qout, qin
                qout[:1].set(np.ones(1, dtype=np.uint32))
                nphotons = int(qin[:1].get()[0]) - 1
                if nphotons == 0:
                    break
        return step_photon_ids, step_photons

    # ---------------------------------------------------------------- selections
    def copy_queue(self, queue_gpu, nphotons, nthreads_per_block=256, max_blocks=1024, start_photon=0):
        out = _alloc(nphotons)
        holder = type('H', (), out)()
        if nphotons > 0:
            _native.call('chr_copy_photon_queue', ctypes.byref(self._desc()), start_photon, nphotons,
                         queue_gpu.gpudata, ctypes.byref(_photons_desc(holder)), current_stream())
        return GPUPhotonsSlice(out['pos'], out['dir'], out['pol'], out['wavelengths'], out['t'],
                               out['last_hit_triangles'], out['flags'], out['weights'], out['evidx'])

    def select(self, target_flag, nthreads_per_block=256, max_blocks=1024, start_photon=None, nphotons=None):
        start = 0 if start_photon is None else start_photon
        n = self.pos.size - start if nphotons is None else nphotons
        count = ctypes.c_uint32()
        desc = self._desc()
        _native.call('chr_select_photons', ctypes.byref(desc), start, n, int(target_flag), None,
                     ctypes.byref(count), current_stream())
        out = _alloc(count.value)
        if count.value:
            holder = type('H', (), out)()
            k = count.value
            _native.call('chr_select_photons', ctypes.byref(desc), start, n, int(target_flag),
                         ctypes.byref(_photons_desc(holder)), ctypes.byref(count), current_stream())
            assert count.value == k
        return GPUPhotonsSlice(out['pos'], out['dir'], out['pol'], out['wavelengths'], out['t'],
                               out['last_hit_triangles'], out['flags'], out['weights'], out['evidx'])


class GPUPhotonsSlice(GPUPhotons):
    """View on GPU photon arrays owned elsewhere (reference photon.py:388-415)."""

    def __init__(self, pos, dir, pol, wavelengths, t, last_hit_triangles, flags, weights, evidx):
        self.pos, self.dir, self.pol = pos, dir, pol
        self.wavelengths, self.t = wavelengths, t
        self.last_hit_triangles, self.flags, self.weights, self.evidx = last_hit_triangles, flags, weights, evidx
        self.true_nphotons = len(pos)
        self.ncopies = 1


def propagate_batches(photon_batches, gpu_geometry, rng_states, nthreads_per_block=256, max_blocks=1024,
                      max_steps=10, use_weights=False, scatter_first=0):
    """Propagate several GPUPhotons in order with one rng_states, as a loop of
    ``gp.propagate(gpu_geometry, rng_states, ...)`` calls would (the event loop
    of Simulation.simulate, reference sim.py:116-160) -- photons and RNG slot
    states end bit-identical -- but pipelined (chr_propagate_batches): batch
    i's multi-step tail, which is as long as its longest-lived photon's serial
    chain, runs on a second HIP stream while batch i+1 is queued, binned and
    walked for its first step.  Each batch's ``last_stats`` is set.  Returns the
    list of stats."""
    batches = list(photon_batches)
    nslots = len(rng_states)
    if nthreads_per_block * max_blocks > nslots:
        raise ValueError('rng_states must have at least nthreads_per_block*max_blocks states')
    nb = len(batches)
    if nb == 0:
        return []
    descs = (_native.PhotonsDesc * nb)(*[gp._desc() for gp in batches])
    n = np.array([gp.pos.size for gp in batches], dtype=np.uint32)
    true_n = np.array([gp.true_nphotons for gp in batches], dtype=np.uint32)
    copies = np.array([gp.ncopies for gp in batches], dtype=np.uint32)
    stats = (_native.PropagateStats * nb)()
    _native.call('chr_propagate_batches', ctypes.c_void_p(gpu_geometry.gpudata), descs, n.ctypes.data,
                 true_n.ctypes.data, copies.ctypes.data, nb, rng_states.gpudata, nslots, nthreads_per_block,
                 max_blocks, max_steps, int(bool(use_weights)), int(scatter_first), stats, current_stream())
    out = []
    for gp, st in zip(batches, stats):
        gp.last_stats = st
        if st.stack_overflows:
            print('WARNING: %d BVH traversals exceeded the 1000-entry stack' % st.stack_overflows, file=sys.stderr)
        out.append(st)
    return out
