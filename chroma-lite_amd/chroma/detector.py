"""Detector = Geometry + PMT channel maps + time/charge response
(drop-in for reference chroma/detector.py:5-140)."""
import numpy as np

from chroma.geometry import Geometry


class Detector(Geometry):
    """A Geometry whose PMT solids are wired to electronics channels.

    Channel indices are 0..nchannels-1 in add_pmt order; channel types are
    arbitrary integers (default: the index).  All channels share one time and
    one charge CDF.
    """

    def __init__(self, detector_material=None):
        Geometry.__init__(self, detector_material=detector_material)
        self.solid_id_to_channel_index = []
        self.channel_index_to_solid_id = []
        self.channel_index_to_channel_type = []
        self.channel_index_to_position = []
        # zero time and unit charge distributions
        self.time_cdf = (np.array([-0.00000001, 0.00000001]), np.array([0.0, 1.0]))
        self.charge_cdf = (np.array([0.999999999, 1.00000000]), np.array([0.0, 1.0]))

    def add_solid(self, solid, rotation=None, displacement=None):
        solid_id = Geometry.add_solid(self, solid=solid, rotation=rotation, displacement=displacement)
        self.solid_id_to_channel_index.append(-1)
        return solid_id

    def add_pmt(self, pmt, rotation=None, displacement=None, channel_type=None):
        solid_id = self.add_solid(solid=pmt, rotation=rotation, displacement=displacement)
        channel_index = len(self.channel_index_to_solid_id)
        if channel_type is None:
            channel_type = channel_index
        self.solid_id_to_channel_index[solid_id] = channel_index
        self.channel_index_to_solid_id.append(solid_id)
        self.channel_index_to_channel_type.append(channel_type)
        self.channel_index_to_position.append(displacement)
        return {'solid_id': solid_id, 'channel_index': channel_index, 'channel_type': channel_type}

    @staticmethod
    def _pdf_to_cdf(bin_edges, bin_contents):
        # NOTE mirrors the reference exactly (detector.py:93-99): there
        # `[0.0] + bin_contents.cumsum()` broadcasts instead of prepending, so
        # cdf_y has len(bin_contents) values while cdf_x has one more.
        cdf_y = np.asarray(bin_contents, dtype=float).cumsum()
        cdf_y = cdf_y / cdf_y[-1]
        return (np.copy(bin_edges), cdf_y)

    def set_time_dist_gaussian(self, rms, lo, hi, nsamples=50):
        x = np.linspace(lo, hi, nsamples + 1, endpoint=True)
        self.time_cdf = self._pdf_to_cdf(x, np.exp(-0.5 * (x[1:] / rms) ** 2))

    def set_time_dist(self, bin_edges, bin_contents):
        self.time_cdf = self._pdf_to_cdf(bin_edges, bin_contents)

    def set_charge_dist_gaussian(self, mean, rms, lo, hi, nsamples=50):
        x = np.linspace(lo, hi, nsamples + 1, endpoint=True)
        self.charge_cdf = self._pdf_to_cdf(x, np.exp(-0.5 * ((x[1:] - mean) / rms) ** 2))

    def num_channels(self):
        return len(self.channel_index_to_channel_type)

    def flatten(self):
        self.solid_id_to_channel_index = np.asarray(self.solid_id_to_channel_index, dtype=np.int32)
        self.channel_index_to_solid_id = np.asarray(self.channel_index_to_solid_id, dtype=np.int32)
        self.channel_index_to_channel_type = np.asarray(self.channel_index_to_channel_type, dtype=np.int32)
        # a PMT added without a displacement sits at the origin (add_pmt's documented
        # default, reference detector.py:60-62); the reference's asarray would raise on None
        self.channel_index_to_position = np.asarray([np.zeros(3) if p is None else p
                                                     for p in self.channel_index_to_position],
                                                    dtype=np.int32).reshape(-1, 3)
        Geometry.flatten(self)
