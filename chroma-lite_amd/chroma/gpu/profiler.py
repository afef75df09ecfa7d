"""Kernel and device-region profiling (drop-in for reference chroma/gpu/profiler.py).

Two layers, as in the reference:

* host side (profiler.py:11-204): per-launch device time of every native
  entry point.  The reference wraps each PyCUDA kernel function; here every
  launch already goes through ``chroma.gpu._native.call``, so ``enable()``
  installs a timer there (HIP events on torch's current stream -- the stream
  every entry point is given -- and a wait on the end event, like the
  reference's ``end.synchronize()``).  ``wrap_function(f, name)`` times any
  other callable the same way.
* device side (profiler.py:207-288): region counters (calls, cycles) of the
  step kernels, compiled into ``libchroma_amd_prof.so`` (the reference's
  ``-DCHROMA_DEVICE_PROFILE=1`` build).  Set ``CHROMA_DEVICE_PROFILE=1`` before
  the first native call to load it; ``device_fetch / device_reset /
  device_report`` then read it (regions: include/chroma_amd.h CHR_PROF_*).

Environment (profiler.py:291-300): ``CHROMA_CUDA_PROFILE=1`` enables the host
profiler at import, ``CHROMA_CUDA_PROFILE_DETAIL=1`` keeps every call's time,
``CHROMA_CUDA_PROFILE_AUTOREPORT=1`` logs the report at exit.
"""
import atexit
import ctypes
import os
import threading
import time

import numpy as np

from chroma.log import logger
from chroma.gpu import _native

# region names by counter index (reference profiler.py:209-214 for 0-3, the rest
# are this build's split kernels; include/chroma_amd.h CHR_PROF_*)
DEVICE_REGION_NAMES = {
    0: 'intersect_mesh',
    1: 'intersect_node',
    2: 'intersect_triangle',
    3: 'intersect_box',
    4: 'fill_material',
    5: 'fill_analytic',
    6: 'trace_refill',
    7: 'trace_idle',
    8: 'shade_physics',
    9: 'shade_other',
    10: 'tail_walk',
    11: 'tail_physics',
    12: 'tail_other',
    13: 'trace_kernel',
    14: 'shade_kernel',
    15: 'tail_kernel',
    16: 'trace_drain',
    17: 'lone_refill',
    18: 'lone_fetch',
    19: 'lone_expand',
    20: 'lone_tris',
    21: 'lone_walk',
    22: 'long_walk',
    23: 'long_fill',
    24: 'long_to_boundary',
    25: 'long_at_boundary',
    26: 'long_other',
}
NREGIONS = 27        # CHR_PROF_NREGIONS
COUNTERS = 64        # CHR_PROF_COUNT (profile.h:16)


class KernelStats:
    """Accumulated device time of one named launch site (ms)."""
    __slots__ = ('name', 'calls', 'total_ms', 'min_ms', 'max_ms', 'last_ms')

    def __init__(self, name):
        self.name = name
        self.calls = 0
        self.total_ms = 0.0
        self.min_ms = float('inf')
        self.max_ms = 0.0
        self.last_ms = 0.0

    def add(self, ms):
        self.calls += 1
        self.total_ms += ms
        self.last_ms = ms
        self.min_ms = min(self.min_ms, ms)
        self.max_ms = max(self.max_ms, ms)

    def as_dict(self):
        return {'calls': self.calls, 'total_ms': self.total_ms,
                'avg_ms': self.total_ms / self.calls if self.calls else 0.0,
                'min_ms': 0.0 if self.calls == 0 else self.min_ms,
                'max_ms': self.max_ms, 'last_ms': self.last_ms}


def _device_timer():
    """(start, stop) -> ms on torch's current HIP stream; wall clock without a device."""
    try:
        import torch
        if torch.cuda.is_available():
            def run(fn):
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                ret = fn()
                e.record()
                e.synchronize()
                return ret, s.elapsed_time(e)
            return run
    except ImportError:
        pass

    def run(fn):
        t0 = time.perf_counter()
        ret = fn()
        return ret, (time.perf_counter() - t0) * 1e3
    return run


class Profiler:
    def __init__(self):
        self._lock = threading.Lock()
        self._enabled = False
        self._detailed = False
        self._stats = {}
        self._per_call = {}
        self._timer = None

    def is_enabled(self):
        return self._enabled

    def enable(self, detailed=False):
        with self._lock:
            self._enabled = True
            self._detailed = detailed
            if self._timer is None:
                self._timer = _device_timer()
            _native.call_hook = self._timed

    def disable(self):
        with self._lock:
            self._enabled = False
            if _native.call_hook == self._timed:
                _native.call_hook = None

    def reset(self):
        with self._lock:
            self._stats.clear()
            self._per_call.clear()

    def _record(self, name, ms):
        with self._lock:
            st = self._stats.get(name)
            if st is None:
                st = self._stats[name] = KernelStats(name)
            st.add(ms)
            if self._detailed:
                self._per_call.setdefault(name, []).append(ms)
                logger.debug('kernel %s took %.3f ms', name, ms)

    def _timed(self, name, fn):
        if not self._enabled:
            return fn()
        ret, ms = self._timer(fn)
        self._record(name, ms)
        return ret

    def wrap_function(self, func, name):
        """A callable that times func(*args, **kwargs) under `name` while enabled."""
        if getattr(func, '_chroma_profiled', False):
            return func
        prof = self

        def wrapped(*args, **kwargs):
            if not prof._enabled:
                return func(*args, **kwargs)
            if prof._timer is None:
                prof._timer = _device_timer()
            return prof._timed(name, lambda: func(*args, **kwargs))
        wrapped._chroma_profiled = True
        wrapped.__wrapped__ = func
        return wrapped

    def per_call(self, name):
        with self._lock:
            return list(self._per_call.get(name, []))

    def stats(self):
        with self._lock:
            return {k: v.as_dict() for k, v in self._stats.items()}

    def report(self, sort_by='total_ms', top=0):
        rows = sorted(self.stats().items(),
                      key=lambda kv: kv[1]['calls' if sort_by == 'calls' else 'total_ms'], reverse=True)
        if top > 0:
            rows = rows[:top]
        lines = ['HIP kernel profile (name | calls | total ms | avg ms | min | max | last):']
        for name, s in rows:
            lines.append('%s | %d | %.3f | %.3f | %.3f | %.3f | %.3f' % (
                name, s['calls'], s['total_ms'], s['avg_ms'], s['min_ms'], s['max_ms'], s['last_ms']))
        text = '\n'.join(lines)
        logger.info(text)
        return text


profiler = Profiler()


def enable(detailed=False):
    profiler.enable(detailed=detailed)


def disable():
    profiler.disable()


def reset():
    profiler.reset()


def is_enabled():
    return profiler.is_enabled()


def wrap_function(func, name):
    return profiler.wrap_function(func, name)


def stats():
    return profiler.stats()


def report(sort_by='total_ms', top=0):
    return profiler.report(sort_by=sort_by, top=top)


# ------------------------------------------------------------ device regions
def device_available():
    """Whether the loaded library carries the device region counters."""
    return bool(_native.lib().chr_device_profile_enabled())


def _require_device_profile():
    if not device_available():
        raise RuntimeError('Device profiling symbols not found: set CHROMA_DEVICE_PROFILE=1 before the first '
                           'native call (loads %s)' % os.path.join(_native._LIBDIR, 'libchroma_amd_prof.so'))


def device_fetch(module=None, n=NREGIONS):
    """{region name: {'calls', 'cycles'}} of the device counters (profiler.py:217-242).
    `module` is accepted for the reference's signature and ignored."""
    _require_device_profile()
    calls = np.zeros(n, dtype=np.uint64)
    cycles = np.zeros(n, dtype=np.uint64)
    khz = ctypes.c_uint32(0)
    _native.call('chr_device_profile_fetch', calls.ctypes.data, cycles.ctypes.data, n, ctypes.byref(khz))
    device_fetch.clock_khz = int(khz.value)
    return {DEVICE_REGION_NAMES.get(i, 'region_%d' % i): {'calls': int(calls[i]), 'cycles': int(cycles[i])}
            for i in range(n)}


device_fetch.clock_khz = 0


def device_reset(module=None):
    """Zero the device counters (profiler.py:245-262)."""
    _require_device_profile()
    from chroma.gpu.tools import current_stream
    _native.call('chr_device_profile_reset', current_stream())


def device_report(module=None, clock_khz=None):
    """Region table in ms (profiler.py:265-288).  cycles are lane-cycles of the
    shader clock (include/chroma_amd.h): total ms is summed over work-items, so
    divide by 64 for wave time."""
    stats = device_fetch(module)
    khz = float(clock_khz or device_fetch.clock_khz or 1000000)
    lines = ['HIP device profile (name | calls | total ms | avg us):']
    for name, s in stats.items():
        total_ms = s['cycles'] / (khz * 1000.0)
        avg_us = total_ms * 1000.0 / s['calls'] if s['calls'] else 0.0
        lines.append('%s | %d | %.3f | %.3f' % (name, s['calls'], total_ms, avg_us))
    text = '\n'.join(lines)
    logger.info(text)
    return text


def _truthy(v):
    return v.strip().lower() in ('1', 'true', 'yes', 'on')


if _truthy(os.environ.get('CHROMA_CUDA_PROFILE', '')):
    enable(detailed=_truthy(os.environ.get('CHROMA_CUDA_PROFILE_DETAIL', '')))
    if _truthy(os.environ.get('CHROMA_CUDA_PROFILE_AUTOREPORT', '')):
        atexit.register(report)
