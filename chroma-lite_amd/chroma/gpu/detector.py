"""GPUDetector (drop-in for reference chroma/gpu/detector.py:14-40): the
geometry plus the solid -> channel map and the shared time/charge CDFs."""
import numpy as np

from chroma.gpu import gpuarray as ga
from chroma.gpu.geometry import GPUGeometry


def cdf_arrays(cdf):
    """(cdf_x, cdf_y) as float32 device-table arrays.  The reference's
    Detector._pdf_to_cdf yields len(cdf_y) == len(cdf_x) - 1 (detector.py:101-102:
    `[0.0] + cumsum` broadcasts instead of prepending), while the kernels take
    len(cdf_x) as the CDF length, so interp reads cdf_y one past its end (UB in
    the reference).  Defined here: cdf_y is padded by repeating its last
    element (1.0 for a normalised CDF)."""
    x = np.asarray(cdf[0], dtype=np.float32)
    y = np.asarray(cdf[1], dtype=np.float32)
    if len(y) < len(x):
        y = np.concatenate([y, np.repeat(y[-1:], len(x) - len(y))])
    return np.ascontiguousarray(x), np.ascontiguousarray(y[:len(x)])


class GPUDetector(GPUGeometry):
    def __init__(self, detector, wavelengths=None, print_usage=False):
        GPUGeometry.__init__(self, detector, wavelengths=wavelengths, print_usage=False)
        self.solid_id_to_channel_index_gpu = ga.to_gpu(np.asarray(detector.solid_id_to_channel_index,
                                                                  dtype=np.int32))
        self.nchannels = detector.num_channels()
        tx, ty = cdf_arrays(detector.time_cdf)
        qx, qy = cdf_arrays(detector.charge_cdf)
        self.time_cdf_x_gpu, self.time_cdf_y_gpu = ga.to_gpu(tx), ga.to_gpu(ty)
        self.charge_cdf_x_gpu, self.charge_cdf_y_gpu = ga.to_gpu(qx), ga.to_gpu(qy)
        self.time_cdf_len = len(tx)      # detector.h time_cdf_len = len(cdf_x) (gpu/detector.py:37)
        self.charge_cdf_len = len(qx)
        self.charge_unit = np.float32(detector.charge_cdf[0][-1] / 2 ** 16)
        self.detector_gpu = self   # kernels take the arrays above directly
