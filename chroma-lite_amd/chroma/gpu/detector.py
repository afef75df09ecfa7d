"""GPUDetector (drop-in for reference chroma/gpu/detector.py:14-40): the
geometry plus the solid -> channel map and the shared time/charge CDFs."""
import numpy as np

from chroma.gpu import gpuarray as ga
from chroma.gpu.geometry import GPUGeometry


class GPUDetector(GPUGeometry):
    def __init__(self, detector, wavelengths=None, print_usage=False):
        GPUGeometry.__init__(self, detector, wavelengths=wavelengths, print_usage=False)
        self.solid_id_to_channel_index_gpu = ga.to_gpu(np.asarray(detector.solid_id_to_channel_index,
                                                                  dtype=np.int32))
        self.nchannels = detector.num_channels()
        self.time_cdf_x_gpu = ga.to_gpu(np.asarray(detector.time_cdf[0], dtype=np.float32))
        self.time_cdf_y_gpu = ga.to_gpu(np.asarray(detector.time_cdf[1], dtype=np.float32))
        self.charge_cdf_x_gpu = ga.to_gpu(np.asarray(detector.charge_cdf[0], dtype=np.float32))
        self.charge_cdf_y_gpu = ga.to_gpu(np.asarray(detector.charge_cdf[1], dtype=np.float32))
        self.charge_unit = np.float32(detector.charge_cdf[0][-1] / 2 ** 16)
        self.detector_gpu = self   # kernels take the arrays above directly
