"""The C-ABI library loads and exports every symbol include/chroma_amd.h declares
(no device calls: runs without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT


def declared_symbols():
    text = open(os.path.join(ROOT, 'include', 'chroma_amd.h')).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(chr_[a-z0-9_]+)\s*\(', text)))


def test_library_exports_all_declared_symbols():
    from chroma.gpu import _native
    lib = ctypes.CDLL(_native.library_path())
    names = declared_symbols()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_native.EXPORTED)


def test_version_and_error_string():
    from chroma.gpu import _native
    l = _native.lib()
    assert l.chr_version() == 1
    assert isinstance(l.chr_last_error(), bytes)


def test_library_built_from_this_tree():
    """The .so travels prebuilt with the tree (the GPU box does not rebuild it):
    the source sha compiled into it (chr_source_sha, csrc/Makefile) must be
    the sha of the sources beside it (tools/source_sha.py)."""
    import sys
    from chroma.gpu import _native
    sys.path.insert(0, os.path.join(ROOT, 'tools'))
    from source_sha import kernel_source_sha
    assert _native.lib().chr_source_sha().decode() == kernel_source_sha(ROOT)


def test_invalid_arguments_fail_loudly():
    import pytest
    from chroma.gpu import _native
    with pytest.raises(_native.NativeError):
        _native.call('chr_bvh_build_grid', None, 0, None, 0, 3, ctypes.byref(ctypes.c_void_p()))
