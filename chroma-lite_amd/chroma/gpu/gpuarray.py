"""A minimal GPU array over torch ROCm tensors.

The reference hands PyCUDA ``gpuarray.GPUArray`` objects around
(chroma/gpu/photon.py:46-62, sim.py:157-223); the drop-in keeps that surface
-- ``get() set() fill() gpudata size nbytes dtype len() [slices]`` and the
``vec.float3/uint3/uint4`` record dtypes -- on top of torch device memory,
which is only storage here (every kernel is ours, launched through the C ABI).
"""
import numpy as np

import torch


class _Vec(object):
    float3 = np.dtype([('x', '<f4'), ('y', '<f4'), ('z', '<f4')])
    float4 = np.dtype([('x', '<f4'), ('y', '<f4'), ('z', '<f4'), ('w', '<f4')])
    uint3 = np.dtype([('x', '<u4'), ('y', '<u4'), ('z', '<u4')])
    uint4 = np.dtype([('x', '<u4'), ('y', '<u4'), ('z', '<u4'), ('w', '<u4')])
    int3 = np.dtype([('x', '<i4'), ('y', '<i4'), ('z', '<i4')])

    @staticmethod
    def make_float3(x, y, z):
        return np.array((x, y, z), dtype=_Vec.float3)


vec = _Vec()

_TORCH = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
          # unsigned words are stored in the same-width signed torch dtype (bit
          # identical; torch's uint32/uint64 kernels are incomplete)
          np.dtype(np.int32): torch.int32, np.dtype(np.uint32): torch.int32,
          np.dtype(np.int64): torch.int64, np.dtype(np.uint64): torch.int64,
          np.dtype(np.uint8): torch.uint8, np.dtype(np.int8): torch.int8, np.dtype(np.bool_): torch.bool}


def _base(dtype):
    """(scalar dtype, components) of a scalar or homogeneous record dtype."""
    dtype = np.dtype(dtype)
    if dtype.names:
        sub = {dtype.fields[n][0] for n in dtype.names}
        assert len(sub) == 1, 'inhomogeneous record dtype %s' % dtype
        return np.dtype(sub.pop()), len(dtype.names)
    return dtype, 1


def _device():
    return torch.device('cuda', torch.cuda.current_device())


class GPUArray(object):
    """1-D array of `dtype` elements in device memory (torch storage)."""

    def __init__(self, shape, dtype, tensor=None):
        self.dtype = np.dtype(dtype)
        self.shape = (int(shape),) if np.isscalar(shape) else tuple(int(s) for s in shape)
        base, k = _base(self.dtype)
        n = int(np.prod(self.shape))
        if tensor is None:
            tensor = torch.empty(n * k, dtype=_TORCH[base], device=_device())
        self._t = tensor            # flat tensor of n*k scalars

    # ---- pycuda-like attributes
    @property
    def size(self):
        return int(np.prod(self.shape))

    @property
    def nbytes(self):
        return self.size * self.dtype.itemsize

    @property
    def gpudata(self):
        return self._t.data_ptr()

    @property
    def ptr(self):
        return self._t.data_ptr()

    @property
    def tensor(self):
        return self._t

    def __len__(self):
        return self.shape[0]

    def __int__(self):
        return self.gpudata

    def get(self):
        host = self._t.cpu().numpy()
        return host.view(self.dtype).reshape(self.shape).copy()

    def set(self, ary):
        ary = np.ascontiguousarray(np.asarray(ary, dtype=self.dtype))
        if ary.size != self.size:
            raise ValueError('size mismatch: %d vs %d' % (ary.size, self.size))
        base, _ = _base(self.dtype)
        flat = ary.reshape(-1).view(base)
        if base.kind == 'u' and base.itemsize in (4, 8):
            flat = flat.view(np.dtype('<i%d' % base.itemsize))
        self._t.copy_(torch.from_numpy(flat))

    def fill(self, value):
        if self.dtype.names:
            raise TypeError('fill() on a vector dtype')
        v = value.item() if isinstance(value, np.generic) else value
        if self.dtype.kind == 'u' and self.dtype.itemsize in (4, 8):
            v = int(np.array(v, dtype=self.dtype).view(np.dtype('<i%d' % self.dtype.itemsize)))
        self._t.fill_(v)
        return self

    def copy(self):
        return GPUArray(self.shape, self.dtype, self._t.clone())

    def __getitem__(self, key):
        if not isinstance(key, slice):
            raise TypeError('GPUArray supports slices only')
        start, stop, step = key.indices(self.shape[0])
        if step != 1:
            raise ValueError('only contiguous slices are supported')
        _, k = _base(self.dtype)
        n = max(0, stop - start)
        return GPUArray((n,), self.dtype, self._t[start * k:(start + n) * k])

    def __repr__(self):
        return 'GPUArray(shape=%s, dtype=%s)' % (self.shape, self.dtype)


def empty(shape, dtype):
    return GPUArray(shape, dtype)


def zeros(shape, dtype):
    a = GPUArray(shape, dtype)
    a._t.zero_()
    return a


def ones_like(other, dtype=None):
    a = GPUArray(other.shape, dtype if dtype is not None else other.dtype)
    a._t.fill_(1)
    return a


def to_gpu(ary):
    ary = np.ascontiguousarray(ary)
    a = GPUArray(ary.shape[:1] if ary.dtype.names else (ary.size,), ary.dtype)
    a.set(ary.reshape(-1) if not ary.dtype.names else ary)
    return a


def from_tensor(tensor, dtype):
    """Wrap an existing device tensor (no copy)."""
    base, k = _base(dtype)
    t = tensor.reshape(-1)
    assert t.dtype == _TORCH[base]
    return GPUArray((t.numel() // k,), dtype, t)
