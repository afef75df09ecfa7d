"""GPURays (drop-in for reference chroma/gpu/render.py:1-66) and the hybrid
renderer's device passes (reference chroma/cuda/hybrid_render.cu, driven by
chroma/camera.py:246-282).

Rays live in device memory as float3 arrays; rendering, the ray transforms
and the hybrid passes are the HIP kernels of csrc/render.hip (C ABI:
chr_render, chr_transform_*, chr_hybrid_*).  Pixel, distance and colour
results are bit-identical to the CPU oracle's restatement of render.cu
(tests/test_gpu_render.py).
"""
import ctypes

import numpy as np

from chroma.gpu import _native
from chroma.gpu import gpuarray as ga
from chroma.gpu.tools import current_stream, to_float3


def _f(x):
    return ctypes.c_float(float(x))


def _vec3(v):
    v = np.asarray(v, dtype=np.float32).reshape(3)
    return [_f(v[0]), _f(v[1]), _f(v[2])]


class GPURays(object):
    """Ray positions and directions on the GPU, used to render a geometry."""

    def __init__(self, pos, dir, max_alpha_depth=10, nblocks=64):
        self.pos = ga.to_gpu(to_float3(pos))
        self.dir = ga.to_gpu(to_float3(dir))
        self.max_alpha_depth = max_alpha_depth
        self.nblocks = nblocks
        self.dx = ga.empty(max_alpha_depth * self.pos.size, dtype=np.float32)
        self.color = ga.empty(self.dx.size, dtype=ga.vec.float4)
        self.dxlen = ga.zeros(self.pos.size, dtype=np.uint32)

    def rotate(self, phi, n):
        """Rotate by an angle phi around the axis `n`."""
        for a in (self.pos, self.dir):
            _native.call('chr_transform_rotate', a.size, a.gpudata, _f(phi), *_vec3(n), current_stream())

    def rotate_around_point(self, phi, n, point):
        """Rotate by an angle phi around the axis `n` passing through the point `point`."""
        _native.call('chr_transform_rotate_around_point', self.pos.size, self.pos.gpudata, _f(phi), *_vec3(n),
                     *_vec3(point), current_stream())
        _native.call('chr_transform_rotate', self.dir.size, self.dir.gpudata, _f(phi), *_vec3(n), current_stream())

    def translate(self, v):
        """Translate the ray positions by the vector `v`."""
        _native.call('chr_transform_translate', self.pos.size, self.pos.gpudata, *_vec3(v), current_stream())

    def render(self, gpu_geometry, pixels, alpha_depth=10, keep_last_render=False, bg_color=0x00000000):
        """Render `gpu_geometry` and fill the GPU array `pixels` with pixel colors."""
        if not keep_last_render:
            self.dxlen.fill(0)
        if alpha_depth > self.max_alpha_depth:
            raise Exception('alpha_depth > max_alpha_depth')
        if not isinstance(pixels, ga.GPUArray):
            raise TypeError('`pixels` must be a %s instance.' % ga.GPUArray)
        if pixels.size != self.pos.size:
            raise ValueError('`pixels`.size != number of rays')
        _native.call('chr_render', gpu_geometry.gpudata, self.pos.size, self.pos.gpudata, self.dir.gpudata,
                     gpu_geometry.colors.gpudata, int(alpha_depth), pixels.gpudata, self.dx.gpudata,
                     self.dxlen.gpudata, self.color.gpudata, ctypes.c_uint32(int(bg_color) & 0xFFFFFFFF),
                     current_stream())

    def snapshot(self, gpu_geometry, alpha_depth=10):
        """Render `gpu_geometry` and return a numpy array of pixel colors."""
        pixels = ga.empty(self.pos.size, dtype=np.uint32)
        self.render(gpu_geometry, pixels, alpha_depth)
        return pixels.get()


def update_xyz_lookup(gpu_geometry, nthreads, total_threads, offset, position, rng_states, wavelength, xyz,
                      lookup1, lookup2, max_steps):
    """hybrid_render.cu update_xyz_lookup: light from `position` to a random
    point of triangle (offset + work-item); its first diffuse reflection adds
    cos_theta * xyz to that triangle's lookup (inside-to-outside: lookup1)."""
    _native.call('chr_hybrid_update_xyz_lookup', gpu_geometry.gpudata, gpu_geometry.vertices.gpudata,
                 gpu_geometry.triangles.gpudata, int(nthreads), int(total_threads), int(offset),
                 (ctypes.c_float * 3)(*[float(x) for x in position]), rng_states.gpudata, rng_states.size,
                 _f(wavelength), (ctypes.c_float * 3)(*[float(x) for x in xyz]), lookup1.gpudata, lookup2.gpudata,
                 int(max_steps), current_stream())


def update_xyz_image(gpu_geometry, rays, rng_states, wavelength, xyz, lookup1, lookup2, image, nlookup_calls,
                     max_steps):
    """hybrid_render.cu update_xyz_image: each ray's first diffuse
    reflection reads the lookup of the triangle it lands on into `image`."""
    _native.call('chr_hybrid_update_xyz_image', gpu_geometry.gpudata, rays.pos.size, rng_states.gpudata,
                 rng_states.size, rays.pos.gpudata, rays.dir.gpudata, _f(wavelength),
                 (ctypes.c_float * 3)(*[float(x) for x in xyz]), lookup1.gpudata, lookup2.gpudata, image.gpudata,
                 int(nlookup_calls), int(max_steps), current_stream())


def process_image(image, pixels, nimages):
    """hybrid_render.cu process_image: average, clamp to [0, 1], pack ARGB."""
    _native.call('chr_hybrid_process_image', pixels.size, image.gpudata, pixels.gpudata, int(nimages),
                 current_stream())
