"""GPUGeometry (drop-in for reference chroma/gpu/geometry.py:13-565).

Packs the geometry (chroma.gpu.packing), obtains the traversal BVH
(chroma.gpu.wide_bvh: cached next to the reference BVH, as the reference
caches the BVH its kernel walks) and uploads both with
chr_geometry_create_wide, which lays them out for the gfx950 traversal kernel
(csrc/device_geometry.h).  `gpudata` is the opaque device-geometry handle the
kernels take.  There is no host-mapped split of the BVH (the reference's
min_free_gpu_mem path, geometry.py:409-439): 288 GB of HBM holds even the
~170 M-triangle 29k-PMT detector many times over.
"""
import ctypes
import time

import numpy as np

from chroma.gpu import _native, wide_bvh
from chroma.gpu import gpuarray as ga
from chroma.gpu.packing import PackedGeometry
from chroma.gpu.tools import format_size
from chroma.log import logger


class GPUGeometry(object):
    def __init__(self, geometry, wavelengths=None, times=None, print_usage=False, min_free_gpu_mem=300e6):
        t0 = time.time()
        if getattr(geometry, 'bvh', None) is None:
            from chroma.loader import load_bvh
            geometry.bvh = load_bvh(geometry)
        self.packed = PackedGeometry(geometry, wavelengths=wavelengths, times=times)
        t1 = time.time()
        # the traversal BVH: attached to the BVH, from the cache next to it, or
        # built on the host (chroma.gpu.wide_bvh); uploaded without a rebuild
        wide, source = wide_bvh.obtain(geometry.bvh, self.packed)
        t2 = time.time()
        handle = ctypes.c_void_p()
        try:
            _native.call('chr_geometry_create_wide', ctypes.byref(self.packed.desc()), ctypes.byref(wide.desc()),
                         ctypes.byref(handle))
        except _native.NativeError as e:
            if source != 'cache':
                raise
            # a cache entry the upload's validation refuses: drop it and build the
            # traversal BVH again, once, instead of failing every run
            # until someone deletes the entry
            logger.warning('traversal BVH from %s refused by the upload (%s): rebuilding', source, e)
            wide_bvh.discard(geometry.bvh)
            wide, source = wide_bvh.obtain(geometry.bvh, self.packed, fresh=True)
            source = 'rebuilt'
            t2 = time.time()
            _native.call('chr_geometry_create_wide', ctypes.byref(self.packed.desc()), ctypes.byref(wide.desc()),
                         ctypes.byref(handle))
        self._handle = handle
        self.geometry = geometry
        self.solid_id_map = ga.to_gpu(np.asarray(geometry.solid_id, dtype=np.uint32))
        self.world_origin = self.packed.world_origin
        self.world_scale = self.packed.world_scale
        # setup phases (bench.py detail.ranks[r].setup): packing the tables / codes,
        # the traversal BVH (cache load or build), the device upload
        self.setup_times = {'pack_s': round(t1 - t0, 3), 'wide_bvh_s': round(t2 - t1, 3), 'wide_bvh_source': source,
                            'h2d_s': round(time.time() - t2, 3)}
        if print_usage:
            self.print_device_usage()
        logger.info(self.device_usage_str())

    @property
    def gpudata(self):
        return self._handle.value

    # The mesh arrays and triangle colours the renderers read (reference
    # geometry.py:389-406 uploads them with the geometry; here on first use,
    # since the propagate path does not need them).
    @property
    def colors(self):
        if getattr(self, '_colors', None) is None:
            colors = getattr(self.geometry, 'colors', None)
            if colors is None or len(colors) != len(self.packed.triangles):
                colors = np.zeros(len(self.packed.triangles), np.uint32)
            self._colors = ga.to_gpu(np.asarray(colors).astype(np.uint32))
        return self._colors

    @property
    def vertices(self):
        if getattr(self, '_vertices', None) is None:
            from chroma.gpu.tools import to_float3
            self._vertices = ga.to_gpu(to_float3(self.packed.vertices))
        return self._vertices

    @property
    def triangles(self):
        if getattr(self, '_triangles', None) is None:
            from chroma.gpu.tools import to_uint3
            self._triangles = ga.to_gpu(to_uint3(self.packed.triangles))
        return self._triangles

    def device_bytes(self):
        b = ctypes.c_uint64()
        _native.call('chr_geometry_device_bytes', self._handle, ctypes.byref(b))
        return b.value

    def phys_words(self):
        """(hot, total) 4-byte words of the physics tables and records
        (chr_geometry_phys_words): the step kernels keep the hot part in LDS
        when it fits (propagate.hip SHADE_PHYS_WORDS / TAIL_PHYS_WORDS)."""
        hot, total = ctypes.c_uint32(), ctypes.c_uint32()
        _native.call('chr_geometry_phys_words', self._handle, ctypes.byref(hot), ctypes.byref(total))
        return hot.value, total.value

    def device_usage_str(self):
        return 'device usage: geometry %s (%d triangles, %d BVH nodes)' % (
            format_size(self.device_bytes()), len(self.packed.triangles), len(self.packed.nodes))

    def print_device_usage(self):
        print(self.device_usage_str())

    def __del__(self):
        h = getattr(self, '_handle', None)
        if h is not None and h.value:
            try:
                _native.lib().chr_geometry_destroy(h)
            except Exception:
                pass
            self._handle = ctypes.c_void_p()
