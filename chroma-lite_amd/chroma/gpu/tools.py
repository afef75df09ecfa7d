"""Device helpers (drop-in for reference chroma/gpu/tools.py).

create_cuda_context selects the HIP device (torch) and returns a context-like
object; get_rng_states allocates the cuRAND-compatible XORWOW slot states and
runs the init kernel (chr_init_rng); chunk_iterator reproduces the reference's
launch chunking exactly (tools.py:159-180), because the RNG slot of a photon
is its index inside a chunk.
"""
import numpy as np
import torch

from chroma.gpu import _native
from chroma.gpu import gpuarray as ga


def current_stream():
    """hipStream_t of torch's current stream, as an int for the C ABI."""
    return torch.cuda.current_stream().cuda_stream


def chunk_iterator(nelements, nthreads_per_block=64, max_blocks=1024):
    """Yield (first_index, elements_this_iteration, nblocks_this_iteration).

    >>> list(chunk_iterator(300, 32, 2))
    [(0, 64, 2), (64, 64, 2), (128, 64, 2), (192, 64, 2), (256, 44, 2)]
    """
    first = 0
    while first < nelements:
        left = nelements - first
        blocks = left // nthreads_per_block + (1 if left % nthreads_per_block else 0)
        blocks = min(max_blocks, blocks)
        count = min(left, blocks * nthreads_per_block)
        yield (first, count, blocks)
        first += count


def to_float3(arr):
    """(N,3) array -> float3 record array."""
    arr = np.ascontiguousarray(arr, dtype=np.float32)
    return arr.view(ga.vec.float3)[:, 0]


def to_uint3(arr):
    arr = np.ascontiguousarray(arr, dtype=np.uint32)
    return arr.view(ga.vec.uint3)[:, 0]


class Context(object):
    """What create_cuda_context returns: the device index plus the two
    methods callers use (pop, synchronize)."""

    def __init__(self, device):
        self.device = device

    def synchronize(self):
        torch.cuda.synchronize(self.device)

    def pop(self):
        self.synchronize()

    def get_current(self):
        return self


def create_cuda_context(device_id=None):
    if not torch.cuda.is_available():
        raise RuntimeError('no HIP device available')
    device = torch.cuda.current_device() if device_id is None else int(device_id)
    torch.cuda.set_device(device)
    _native.lib()
    return Context(device)


class RNGStates(object):
    """`size` XORWOW slot states (6 x u32, SoA) in device memory."""

    def __init__(self, size):
        self.size = int(size)
        self.array = ga.empty(6 * self.size, np.uint32)

    @property
    def gpudata(self):
        return self.array.gpudata

    def __len__(self):
        return self.size

    def get(self):
        """Host copy, shape (6, size): rows d, v0..v4."""
        return self.array.get().reshape(6, self.size)

    @property
    def normal_cache(self):
        """curand_normal's cached second value per slot ({flag, bits}, 2 x u32
        SoA; zero = empty, as curand_init leaves it).  Allocated on first use
        (only the ndaq > 1 DAQ draws normals)."""
        if getattr(self, '_normal', None) is None:
            self._normal = ga.zeros(2 * self.size, np.uint32)
        return self._normal


def get_rng_states(size, seed=1, offset=0, first_subsequence=0):
    """Return `size` random-number-generator states, slot s initialised as
    curand_init(seed, first_subsequence + s, offset).  first_subsequence is an
    extension for photon-sharded runs (rank r of a job takes subsequences
    [r*size, (r+1)*size) so no two ranks share a stream); 0 is the reference."""
    st = RNGStates(size)
    if first_subsequence:
        _native.call('chr_init_rng_subseq', st.gpudata, st.size, int(seed) & (2 ** 64 - 1), int(first_subsequence),
                     int(offset), current_stream())
    else:
        _native.call('chr_init_rng', st.gpudata, st.size, int(seed) & (2 ** 64 - 1), int(offset), current_stream())
    return st


def format_size(size):
    for div, unit in ((1, ' '), (1e3, 'K'), (1e6, 'M'), (1e9, 'G')):
        if size < div * 1e3 or unit == 'G':
            return '%.1f%s' % (size / div, unit)


def format_array(name, array):
    return '%-15s %6s %6s' % (name, format_size(len(array)), format_size(array.nbytes))
