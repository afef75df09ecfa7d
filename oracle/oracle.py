"""TEST INFRASTRUCTURE ONLY: ctypes front-end of the CPU oracle (liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
The product never imports it.  See chroma_oracle.c for what is restated from
the reference and how parity is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBPATH = os.path.join(HERE, '_build', 'liboracle.so')
_lib = None


def build():
    subprocess.check_call(['make', '-s', '-C', HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIBPATH):
            build()
        l = ctypes.CDLL(LIBPATH)
        vp, u32, i32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_ulonglong
        l.orc_rng_init.argtypes = [vp, u32, u64, u64]
        l.orc_rng_init_subseq.argtypes = [vp, u32, u64, u64, u64]
        l.orc_daq.argtypes = [vp] * 8 + [i32, vp, vp, i32, ctypes.c_float, vp, u32, vp, u32, i32, i32,
                                         vp, vp, vp, i32, i32, ctypes.c_float, i32, i32]
        l.orc_sequence_matrices.argtypes = [vp, i32]
        l.orc_rng_uniforms.argtypes = [vp, u32, u32, i32, vp]
        l.orc_distance_to_mesh.argtypes = [vp, i32, vp, vp, vp, vp, vp]
        l.orc_propagate.argtypes = [vp] + [vp] * 9 + [u32, u32, u32, vp, u32, i32, i32, i32, i32, i32, i32, vp]
        l.orc_fill_state.argtypes = [vp, vp, ctypes.c_int32, ctypes.c_float, vp, vp]
        l.orc_math.argtypes = [i32, i32, vp, vp, vp]
        l.orc_rayleigh.argtypes = [i32, vp, vp, vp, u32]
        l.orc_render.argtypes = [vp, i32, vp, vp, vp, u32, vp, vp, vp, vp, u32]
        l.orc_transform.argtypes = [i32, vp, i32, ctypes.c_float, vp, vp]
        l.orc_hybrid_update_xyz_lookup.argtypes = [vp, i32, i32, i32, vp, vp, u32, ctypes.c_float, vp, vp, vp, i32]
        l.orc_hybrid_update_xyz_image.argtypes = [vp, i32, vp, u32, vp, vp, ctypes.c_float, vp, vp, vp, vp, i32, i32]
        l.orc_hybrid_process_image.argtypes = [i32, vp, vp, i32]
        l.orc_set_watch.argtypes = [ctypes.c_int64, vp, u32]
        l.orc_watch_count.restype = u32
        l.orc_intersect_rays.argtypes = [vp, i32, vp, vp, vp, vp, vp]
        l.orc_undershoot.argtypes = [vp]
        _lib = l
    return _lib


def _p(a):
    return a.ctypes.data if a is not None else None


def rng_init(nslots, seed=1, offset=0, first_subsequence=0):
    st = np.zeros(6 * nslots, dtype=np.uint32)
    lib().orc_rng_init_subseq(_p(st), nslots, seed, first_subsequence, offset)
    return st


def sequence_matrices(nlevels):
    out = np.zeros(nlevels * 800, dtype=np.uint32)
    lib().orc_sequence_matrices(_p(out), nlevels)
    return out.reshape(nlevels, 800)


def uniforms(states, nslots, slot, n):
    out = np.zeros(n, dtype=np.float32)
    lib().orc_rng_uniforms(_p(states), nslots, slot, n, _p(out))
    return out


MATH = {'log': 0, 'exp': 1, 'sin': 2, 'cos': 3, 'tan': 4, 'asin': 5, 'acos': 6, 'atan2': 7}


def math(name, x, y=None):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.ascontiguousarray(y if y is not None else np.zeros_like(x), dtype=np.float32)
    out = np.zeros_like(x)
    lib().orc_math(MATH[name], len(x), _p(x), _p(y), _p(out))
    return out


def distance_to_mesh(packed, origins, directions):
    o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(directions, dtype=np.float32).reshape(-1, 3)
    dist = np.zeros(len(o), dtype=np.float32)
    tri = np.zeros(len(o), dtype=np.int32)
    counts = np.zeros(2, dtype=np.uint64)
    desc = packed.desc()
    lib().orc_distance_to_mesh(ctypes.addressof(desc), len(o), _p(o), _p(d), _p(dist), _p(tri), _p(counts))
    return dist, tri, counts


def intersect_rays(packed, origins, directions, last_hit):
    """The reference DFS walk of rays exactly as given (no normalisation) with
    their last-hit triangles: (distance, triangle) per ray."""
    o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
    d = np.ascontiguousarray(directions, dtype=np.float32).reshape(-1, 3)
    last = np.ascontiguousarray(last_hit, dtype=np.int32)
    dist = np.zeros(len(o), dtype=np.float32)
    tri = np.zeros(len(o), dtype=np.int32)
    desc = packed.desc()
    lib().orc_intersect_rays(ctypes.addressof(desc), len(o), _p(o), _p(d), _p(last), _p(dist), _p(tri))
    return dist, tri


def undershoot():
    """(count, max absolute, max relative) of Moller-Trumbore hits before their
    own reference leaf box's entry distance since the last call (diagnostic)."""
    out = np.zeros(3, np.float64)
    lib().orc_undershoot(_p(out))
    return int(out[0]), float(out[1]), float(out[2])


class HostPhotons(object):
    """Writable host copies of the nine photon arrays (float3 as (n,3))."""
    FIELDS = ('pos', 'dir', 'pol', 'wavelengths', 't', 'flags', 'last_hit_triangles', 'weights', 'evidx')
    DTYPES = (np.float32, np.float32, np.float32, np.float32, np.float32, np.uint32, np.int32, np.float32, np.uint32)

    def __init__(self, photons):
        for f, dt in zip(self.FIELDS, self.DTYPES):
            setattr(self, f, np.array(getattr(photons, f), dtype=dt, copy=True, order='C'))

    def __len__(self):
        return len(self.pos)


def propagate(packed, photons, rng_states, nslots, nthreads_per_block=256, max_blocks=1024, max_steps=10,
              use_weights=False, scatter_first=0, ncopies=1, true_nphotons=None, threads=None):
    """GPUPhotons.propagate semantics on the host; photons (HostPhotons) and
    rng_states are updated in place.  Returns the oracle's stats dict."""
    n = len(photons)
    true_n = n // ncopies if true_nphotons is None else true_nphotons
    stats = np.zeros(8, dtype=np.uint64)
    threads = threads or os.cpu_count() or 1
    desc = packed.desc()
    rc = lib().orc_propagate(ctypes.addressof(desc), _p(photons.pos), _p(photons.dir), _p(photons.pol),
                             _p(photons.wavelengths), _p(photons.t), _p(photons.flags),
                             _p(photons.last_hit_triangles), _p(photons.weights), _p(photons.evidx),
                             n, true_n, ncopies, _p(rng_states), nslots, nthreads_per_block, max_blocks,
                             max_steps, int(bool(use_weights)), int(scatter_first), threads, _p(stats))
    if rc != 0:
        raise RuntimeError('orc_propagate failed with status %d' % rc)
    keys = ('nodes_visited', 'tris_tested', 'max_depth', 'overflows', 'host_steps', 'launches', 'final_alive',
            'traversals')
    return dict(zip(keys, (int(x) for x in stats[:8])))


class Watch(object):
    """Every step of one photon (its index in the batch propagate() is given)
    recorded by the oracle: 20 words per step (chroma_oracle.c orc_set_watch,
    the layout of the HIP library's chr_watch_fetch)."""

    def __init__(self, photon, cap=4096):
        self.buf = np.zeros((cap, 20), dtype=np.uint32)
        lib().orc_set_watch(int(photon), _p(self.buf), cap)

    def records(self):
        n = min(int(lib().orc_watch_count()), len(self.buf))
        return self.buf[:n].copy()

    @staticmethod
    def off():
        lib().orc_set_watch(-1, None, 0)


def fill_state(packed, pos, dir, last_hit=-1, wavelength=400.0):
    pd = np.ascontiguousarray(np.concatenate([pos, dir]), dtype=np.float32)
    out = np.zeros(8, dtype=np.float32)
    iout = np.zeros(4, dtype=np.int32)
    desc = packed.desc()
    lib().orc_fill_state(ctypes.addressof(desc), _p(pd), int(last_hit), float(wavelength), _p(out), _p(iout))
    return out, iout


def rayleigh(dir, pol, states, nslots):
    d = np.ascontiguousarray(dir, dtype=np.float32).copy()
    p = np.ascontiguousarray(pol, dtype=np.float32).copy()
    lib().orc_rayleigh(len(d), _p(d), _p(p), _p(states), nslots)
    return d, p


# ---- numpy restatements of the selection kernels (propagate.cu:29-251),
# ascending photon order (the reference's warp-atomic order is arbitrary)
def hits(photons, solid_id, solid_id_to_channel_index, detection_state=0x4, start=0, n=None):
    n = len(photons) - start if n is None else n
    sl = slice(start, start + n)
    tri = np.asarray(photons.last_hit_triangles[sl])
    flagged = (np.asarray(photons.flags[sl]) & detection_state) != 0
    ok = flagged & (tri > -1)
    channel = np.full(n, -1, dtype=np.int32)
    channel[ok] = np.asarray(solid_id_to_channel_index)[np.asarray(solid_id)[tri[ok]]]
    sel = ok & (channel >= 0)
    return np.flatnonzero(sel) + start, channel[sel]


def select(photons, target_flag, start=0, n=None):
    n = len(photons) - start if n is None else n
    return np.flatnonzero((np.asarray(photons.flags[start:start + n]) & target_flag) != 0) + start


def daq(photons, solid_id, solid_id_to_channel_index, time_cdf, charge_cdf, charge_unit, rng_states, nslots,
        normal_cache=None, start=0, n=None, ndaq=1, nchannels=None, global_weight=1.0, nthreads_per_block=64,
        max_blocks=1024, detection_state=0x4, maxtime=1e9, raw=False):
    """GPUDaq begin/acquire/end (daq.py:56-101) on the host.  time_cdf /
    charge_cdf are the (x, y) arrays as the device holds them (equal lengths).
    rng_states / normal_cache are updated in place.  Returns (t, q, flags),
    each of ndaq*nchannels entries (raw=True: the u32 words before end_acquire)."""
    n = len(photons) - start if n is None else n
    nchannels = int(nchannels)
    total = nchannels * ndaq
    time_int = np.full(total, np.float32(maxtime).view(np.uint32), dtype=np.uint32)
    q_int = np.zeros(total, dtype=np.uint32)
    hist = np.zeros(total, dtype=np.uint32)
    if normal_cache is None:
        normal_cache = np.zeros(2 * nslots, dtype=np.uint32)
    a = [np.ascontiguousarray(x, dtype=np.float32) for x in (time_cdf[0], time_cdf[1], charge_cdf[0], charge_cdf[1])]
    sm = np.ascontiguousarray(solid_id, dtype=np.uint32)
    s2c = np.ascontiguousarray(solid_id_to_channel_index, dtype=np.int32)
    rc = lib().orc_daq(_p(photons.t), _p(photons.flags), _p(photons.last_hit_triangles), _p(photons.weights),
                       _p(sm), _p(s2c), _p(a[0]), _p(a[1]), len(a[0]), _p(a[2]), _p(a[3]), len(a[2]),
                       float(charge_unit), _p(rng_states), nslots, _p(normal_cache), detection_state, start, n,
                       _p(time_int), _p(q_int), _p(hist), ndaq, nchannels, float(global_weight),
                       nthreads_per_block, max_blocks)
    if rc != 0:
        raise RuntimeError('orc_daq failed with status %d' % rc)
    if raw:          # the u32 accumulator words (time bits, quantised charge, history)
        return time_int, q_int, hist
    t = time_int.view(np.float32).copy()
    q = np.zeros(total, dtype=np.float32)
    q[:nchannels] = q_int[:nchannels].astype(np.float32) * np.float32(charge_unit)
    return t, q, hist


# ------------------------------------------------------------------ PDF (pdf_oracle.c)
def _pdf_lib():
    l = lib()
    if not getattr(l, '_pdf_bound', False):
        vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        l.orc_pdf_bin_hits.argtypes = [i32, vp, vp, vp, i32, f32, f32, i32, f32, f32, vp]
        l.orc_pdf_accumulate_bincount.argtypes = [i32, i32, vp, vp, vp, vp, vp, f32, f32, f32, i32, vp, vp]
        l.orc_pdf_accumulate_nearest.argtypes = [i32, i32, vp, vp, vp, vp, vp, i32]
        l.orc_pdf_accumulate_moments.argtypes = [i32, i32, vp, vp, f32, f32, f32, f32, vp, vp, vp, vp, vp]
        l.orc_pdf_accumulate_kernel_eval.argtypes = [i32, i32, vp, vp, vp, vp, vp, f32, f32, f32, f32, vp, vp,
                                                     vp, vp, vp]
        l.orc_erff.argtypes = [i32, vp, vp]
        l._pdf_bound = True
    return l


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def erff(x):
    x = _f32(x)
    y = np.zeros_like(x)
    _pdf_lib().orc_erff(len(x), _p(x), _p(y))
    return y


def pdf_bin_hits(q, t, hitcount, pdf, tbins, trange, qbins, qrange):
    """bin_hits (pdf.cu:9-32); hitcount / pdf (u32) updated in place."""
    q, t = _f32(q), _f32(t)
    _pdf_lib().orc_pdf_bin_hits(len(hitcount), _p(q), _p(t), _p(hitcount), tbins, trange[0], trange[1], qbins,
                                qrange[0], qrange[1], _p(pdf))


def pdf_accumulate_bincount(event_hit, event_time, mc_time, ndaq, hitcount, bincount, work_queues, min_twidth,
                            trange, min_bin_content, map_channel_to_hit):
    """accumulate_bincount (pdf.cu:34-96); hitcount / bincount / work_queues in place."""
    eh, et, mt, m = _u32(event_hit), _f32(event_time), _f32(mc_time), _u32(map_channel_to_hit)
    _pdf_lib().orc_pdf_accumulate_bincount(len(eh), ndaq, _p(eh), _p(et), _p(mt), _p(hitcount), _p(bincount),
                                           min_twidth, trange[0], trange[1], min_bin_content, _p(m),
                                           _p(work_queues))


def pdf_accumulate_nearest(map_hit_to_channel, work_queues, event_time, mc_time, ndaq, nearest_mc, min_bin_content):
    """accumulate_nearest_neighbor (pdf.cu:98-150); nearest_mc in place."""
    m, et, mt = _u32(map_hit_to_channel), _f32(event_time), _f32(mc_time)
    _pdf_lib().orc_pdf_accumulate_nearest(len(m), ndaq, _p(m), _p(work_queues), _p(et), _p(mt), _p(nearest_mc),
                                          min_bin_content)


def pdf_accumulate_moments(time_only, mc_time, mc_charge, trange, qrange, mom0, tm1, tm2, qm1, qm2):
    """accumulate_moments (pdf.cu:223-266); accumulators in place."""
    mt, mq = _f32(mc_time), _f32(mc_charge)
    _pdf_lib().orc_pdf_accumulate_moments(int(time_only), len(mom0), _p(mt), _p(mq), trange[0], trange[1], qrange[0],
                                          qrange[1], _p(mom0), _p(tm1), _p(tm2), _p(qm1), _p(qm2))


def pdf_accumulate_kernel_eval(time_only, event_hit, event_time, event_charge, mc_time, mc_charge, trange, qrange,
                               inv_tbw, inv_qbw, hitcount, time_pdf, charge_pdf):
    """accumulate_kernel_eval (pdf.cu:271-368); accumulators in place."""
    eh, et, eq = _u32(event_hit), _f32(event_time), _f32(event_charge)
    mt, mq, it, iq = _f32(mc_time), _f32(mc_charge), _f32(inv_tbw), _f32(inv_qbw)
    _pdf_lib().orc_pdf_accumulate_kernel_eval(int(time_only), len(eh), _p(eh), _p(et), _p(eq), _p(mt), _p(mq),
                                              trange[0], trange[1], qrange[0], qrange[1], _p(it), _p(iq),
                                              _p(hitcount), _p(time_pdf), _p(charge_pdf))


# ---------------------------------------------------------------- renderer
def render(packed, pos, dir, colors, alpha_depth, dx=None, dxlen=None, color=None, bg_color=0):
    """render.cu:37-183 restated (reference BVH, reference order, searchsorted
    insertion).  Returns (pixels, dx, dxlen, color); pass dx/dxlen/color of a
    previous call to merge (keep_last_render)."""
    pos = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
    dir = np.ascontiguousarray(dir, np.float32).reshape(-1, 3)
    n = len(pos)
    colors = np.ascontiguousarray(colors, np.uint32)
    dx = np.zeros(n * alpha_depth, np.float32) if dx is None else dx
    dxlen = np.zeros(n, np.uint32) if dxlen is None else dxlen
    color = np.zeros(n * alpha_depth * 4, np.float32) if color is None else color
    pixels = np.zeros(n, np.uint32)
    desc = packed.desc()
    rc = lib().orc_render(ctypes.addressof(desc), n, _p(pos), _p(dir), _p(colors), alpha_depth, _p(pixels), _p(dx),
                          _p(dxlen), _p(color), int(bg_color) & 0xFFFFFFFF)
    if rc != 0:
        raise RuntimeError('orc_render failed with status %d' % rc)
    return pixels, dx, dxlen, color


def transform(a, mode, phi=0.0, axis=(0, 0, 1), v=(0, 0, 0)):
    """transform.cu: mode 0 translate by v, 1 rotate(phi, axis), 2 rotate about point v."""
    a = np.ascontiguousarray(a, np.float32).reshape(-1, 3).copy()
    ax = np.asarray(axis, np.float32)
    vv = np.asarray(v, np.float32)
    lib().orc_transform(len(a), _p(a), mode, float(phi), _p(ax), _p(vv))
    return a


def hybrid_update_xyz_lookup(packed, nthreads, total_threads, offset, position, rng_states, nslots, wavelength, xyz,
                             lookup1, lookup2, max_steps):
    p = np.asarray(position, np.float32)
    w = np.asarray(xyz, np.float32)
    desc = packed.desc()
    lib().orc_hybrid_update_xyz_lookup(ctypes.addressof(desc), nthreads, total_threads, offset, _p(p), _p(rng_states),
                                       nslots, float(wavelength), _p(w), _p(lookup1), _p(lookup2), max_steps)


def hybrid_update_xyz_image(packed, pos, dir, rng_states, nslots, wavelength, xyz, lookup1, lookup2, image,
                            nlookup_calls, max_steps):
    pos = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
    dir = np.ascontiguousarray(dir, np.float32).reshape(-1, 3)
    w = np.asarray(xyz, np.float32)
    desc = packed.desc()
    lib().orc_hybrid_update_xyz_image(ctypes.addressof(desc), len(pos), _p(rng_states), nslots, _p(pos), _p(dir),
                                      float(wavelength), _p(w), _p(lookup1), _p(lookup2), _p(image), nlookup_calls,
                                      max_steps)


def hybrid_process_image(image, nimages):
    image = np.ascontiguousarray(image, np.float32)
    pixels = np.zeros(len(image) // 3, np.uint32)
    lib().orc_hybrid_process_image(len(pixels), _p(image), _p(pixels), nimages)
    return pixels
