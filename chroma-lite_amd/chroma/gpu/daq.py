"""GPUDaq / GPUChannels (drop-in for reference chroma/gpu/daq.py:8-101).

The DAQ turns detected photons into per-channel readout: earliest time
(photon time + a sample of the detector's time CDF), integrated charge (a
sample of the charge CDF, quantised by charge_unit) and the OR of the photon
histories.  Kernels: csrc/daq.hip through the C ABI (chr_daq_begin /
chr_daq_acquire / chr_daq_end); no host fallback.
"""
import ctypes

import numpy as np

from chroma import event
from chroma.gpu import _native
from chroma.gpu import gpuarray as ga
from chroma.gpu.tools import current_stream


class GPUChannels(object):
    """Per-channel device arrays t (f32), q (f32), flags (u32); ndaq copies of
    `stride` channels each (daq.py:8-36)."""

    def __init__(self, t, q, flags, ndaq=1, stride=None):
        self.t = t
        self.q = q
        self.flags = flags
        self.ndaq = ndaq
        self.stride = len(t) if stride is None else stride

    def iterate_copies(self):
        for i in range(self.ndaq):
            w = slice(i * self.stride, (i + 1) * self.stride)
            yield GPUChannels(self.t[w], self.q[w], self.flags[w])

    def get(self):
        t = self.t.get()
        q = self.q.get()
        # a channel counts as hit when its earliest time is below 1e8 (daq.py:32-34)
        return event.Channels(t < 1e8, t, q, self.flags.get())

    def __len__(self):
        return self.t.size


class _DetectorDesc(ctypes.Structure):   # chr_daq_detector (include/chroma_amd.h)
    _fields_ = [('d_solid_id_to_channel_index', ctypes.c_void_p), ('d_time_cdf_x', ctypes.c_void_p),
                ('d_time_cdf_y', ctypes.c_void_p), ('d_charge_cdf_x', ctypes.c_void_p),
                ('d_charge_cdf_y', ctypes.c_void_p), ('nchannels', ctypes.c_int32), ('time_cdf_len', ctypes.c_int32),
                ('charge_cdf_len', ctypes.c_int32), ('charge_unit', ctypes.c_float)]


def detector_desc(gpu_detector):
    """chr_daq_detector for a GPUDetector (the reference's Detector struct,
    gpu/detector.py:29-40)."""
    return _DetectorDesc(gpu_detector.solid_id_to_channel_index_gpu.gpudata, gpu_detector.time_cdf_x_gpu.gpudata,
                         gpu_detector.time_cdf_y_gpu.gpudata, gpu_detector.charge_cdf_x_gpu.gpudata,
                         gpu_detector.charge_cdf_y_gpu.gpudata, int(gpu_detector.nchannels),
                         int(gpu_detector.time_cdf_len), int(gpu_detector.charge_cdf_len),
                         float(gpu_detector.charge_unit))


class GPUDaq(object):
    def __init__(self, gpu_detector, ndaq=1):
        assert gpu_detector.nchannels > 0, "Geometry has no detectors, DAQ can't be initialized."
        n = gpu_detector.nchannels * ndaq
        self.earliest_time_gpu = ga.empty(n, np.float32)
        self.earliest_time_int_gpu = ga.empty(n, np.uint32)
        self.channel_history_gpu = ga.zeros(n, np.uint32)
        self.channel_q_int_gpu = ga.zeros(n, np.uint32)
        self.channel_q_gpu = ga.zeros(n, np.float32)
        self.detector_gpu = gpu_detector.detector_gpu
        self.solid_id_map_gpu = gpu_detector.solid_id_map
        self.solid_id_to_channel_index_gpu = gpu_detector.solid_id_to_channel_index_gpu
        self._desc = detector_desc(gpu_detector)
        self.charge_unit = float(gpu_detector.charge_unit)
        self.nchannels = int(gpu_detector.nchannels)
        self.ndaq = ndaq
        self.stride = gpu_detector.nchannels

    def begin_acquire(self, nthreads_per_block=64):
        """daq.py:56-60: earliest times = 1e9, charges and histories = 0."""
        _native.call('chr_daq_begin', self.earliest_time_int_gpu.gpudata, self.channel_q_int_gpu.gpudata,
                     self.channel_history_gpu.gpudata, len(self.earliest_time_int_gpu), ctypes.c_float(1e9),
                     current_stream())
        self.channel_q_gpu.fill(0)

    def acquire(self, gpuphotons, rng_states, nthreads_per_block=64, max_blocks=1024, start_photon=None,
                nphotons=None, weight=1.0):
        """daq.py:62-91 (run_daq for ndaq == 1, run_daq_many otherwise)."""
        start = 0 if start_photon is None else int(start_photon)
        n = len(gpuphotons.pos) - start if nphotons is None else int(nphotons)
        ph = gpuphotons._desc()
        normal = rng_states.normal_cache.gpudata if self.ndaq > 1 else None
        _native.call('chr_daq_acquire', ctypes.byref(ph), rng_states.gpudata, len(rng_states), normal,
                     0x1 << 2, start, n, self.solid_id_map_gpu.gpudata, ctypes.byref(self._desc),
                     self.earliest_time_int_gpu.gpudata, self.channel_q_int_gpu.gpudata,
                     self.channel_history_gpu.gpudata, int(self.ndaq), int(self.stride), ctypes.c_float(weight),
                     int(nthreads_per_block), int(max_blocks), current_stream())

    def end_acquire(self, nthreads_per_block=64):
        """daq.py:93-101: times back to float, charges * charge_unit."""
        _native.call('chr_daq_end', self.earliest_time_int_gpu.gpudata, self.earliest_time_gpu.gpudata,
                     self.channel_q_int_gpu.gpudata, self.channel_q_gpu.gpudata, len(self.earliest_time_int_gpu),
                     self.nchannels, ctypes.c_float(self.charge_unit), current_stream())
        return GPUChannels(self.earliest_time_gpu, self.channel_q_gpu, self.channel_history_gpu, self.ndaq,
                           self.stride)
