"""Host-side kernel profiler (reference chroma/gpu/profiler.py:11-204) and the
device-profile library's exports; no device calls."""
import ctypes
import os

import pytest

from test_native_abi import declared_symbols


def test_wrap_function_and_report():
    from chroma.gpu import profiler
    p = profiler.Profiler()
    f = p.wrap_function(lambda x: x + 1, 'incr')
    assert f(1) == 2                      # disabled: passes through, nothing recorded
    assert p.stats() == {}
    p.enable(detailed=True)
    assert f(2) == 3 and f(3) == 4
    s = p.stats()['incr']
    assert s['calls'] == 2 and s['min_ms'] <= s['avg_ms'] <= s['max_ms'] and s['last_ms'] >= 0.0
    assert len(p.per_call('incr')) == 2
    assert p.wrap_function(f, 'again') is f
    text = p.report(sort_by='calls', top=1)
    assert text.splitlines()[1].startswith('incr | 2 |')
    p.reset()
    assert p.stats() == {}
    p.disable()


def test_enable_times_native_calls():
    from chroma.gpu import _native, profiler
    profiler.reset()
    profiler.enable()
    try:
        assert _native.call_hook is not None
        _native.call('chr_device_profile_enabled')      # status 0 from the default build
        with pytest.raises(_native.NativeError):      # errors still raise through the hook
            _native.call('chr_bvh_build_grid', None, 0, None, 0, 3, ctypes.byref(ctypes.c_void_p()))
        st = profiler.stats()
        assert st['chr_device_profile_enabled']['calls'] == 1
        assert 'chr_bvh_build_grid' not in st          # a failed launch is not timed (as the reference)
    finally:
        profiler.disable()
        profiler.reset()
    assert _native.call_hook is None


def test_default_build_has_no_device_counters():
    from chroma.gpu import _native, profiler
    if _native.DEVICE_PROFILE:
        pytest.skip('CHROMA_DEVICE_PROFILE set for this process')
    assert not profiler.device_available()
    with pytest.raises(RuntimeError, match='CHROMA_DEVICE_PROFILE'):
        profiler.device_fetch()
    with pytest.raises(_native.NativeError):
        _native.call('chr_device_profile_reset', None)


def test_profile_library_exports():
    from chroma.gpu import _native
    path = os.path.join(_native._LIBDIR, 'libchroma_amd_prof.so')
    lib = ctypes.CDLL(path)
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.chr_device_profile_enabled() == 1
    assert lib.chr_version() == 1
    names = __import__('chroma.gpu.profiler', fromlist=['x']).DEVICE_REGION_NAMES
    assert len(names) == 27 and names[0] == 'intersect_mesh' and names[3] == 'intersect_box'
    assert names[21] == 'lone_walk' and names[26] == 'long_other'
