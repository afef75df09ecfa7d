"""GPUPDF / GPUKernelPDF (drop-in for reference chroma/gpu/pdf.py:7-372).

Per-channel hit-time / charge PDFs built from DAQ output (GPUChannels):
histograms (GPUPDF.setup_pdf / add_hits_to_pdf / get_pdfs), the adaptive
nearest-neighbour evaluation at one event (setup_pdf_eval /
accumulate_pdf_eval / get_pdf_eval) and the Gaussian kernel-density estimate
(GPUKernelPDF).  The device passes are csrc/pdf.hip through the C ABI
(chr_pdf_*); the small host steps (bandwidth choice, final normalisation)
are numpy, as in the reference.  No host fallback for the device passes.
"""
import ctypes

import numpy as np

from chroma.gpu import _native
from chroma.gpu import gpuarray as ga
from chroma.gpu.tools import current_stream

_f = ctypes.c_float


def _channel_words(gpuchannels, n):
    if len(gpuchannels.t) < n:
        raise ValueError('GPUChannels hold %d words, %d channels expected' % (len(gpuchannels.t), n))
    return gpuchannels.t.gpudata, gpuchannels.q.gpudata


class GPUKernelPDF(object):
    """Kernel-density PDF values at one event (pdf.py:7-175)."""

    def setup_moments(self, nchannels, trange, qrange, time_only=True):
        """pdf.py:13-32: per-channel MC moments for the bandwidth choice."""
        self.hitcount_gpu = ga.zeros(nchannels, np.uint32)
        self.tmom1_gpu = ga.zeros(nchannels, np.float32)
        self.tmom2_gpu = ga.zeros(nchannels, np.float32)
        self.qmom1_gpu = ga.zeros(nchannels, np.float32)
        self.qmom2_gpu = ga.zeros(nchannels, np.float32)
        self.trange = trange
        self.qrange = qrange
        self.time_only = time_only

    def clear_moments(self):
        for a in (self.hitcount_gpu, self.tmom1_gpu, self.tmom2_gpu, self.qmom1_gpu, self.qmom2_gpu):
            a.fill(0)

    def accumulate_moments(self, gpuchannels, nthreads_per_block=64):
        """pdf.py:42-59 -> accumulate_moments (pdf.cu:223-266)."""
        n = len(self.hitcount_gpu)
        t, q = _channel_words(gpuchannels, n)
        _native.call('chr_pdf_accumulate_moments', int(bool(self.time_only)), n, t, q, _f(self.trange[0]),
                     _f(self.trange[1]), _f(self.qrange[0]), _f(self.qrange[1]), self.hitcount_gpu.gpudata,
                     self.tmom1_gpu.gpudata, self.tmom2_gpu.gpudata, self.qmom1_gpu.gpudata, self.qmom2_gpu.gpudata,
                     current_stream())

    def compute_bandwidth(self, event_hit, event_time, event_charge, scale_factor=1.0):
        """pdf.py:61-112: Silverman-style bandwidth per channel from the moments."""
        rho = 1.0
        mom0 = np.maximum(self.hitcount_gpu.get(), 1)
        d = 1 if self.time_only else 2
        dim_factor = ((4.0 / (d + 2)) / (mom0 / scale_factor)) ** (-1.0 / (d + 4))

        def bandwidth(mom1, mom2, obs, clip_negative_variance):
            mean = mom1 / mom0
            var = mom2 / mom0 - mean ** 2
            rms = (np.maximum(var, 0.0) if clip_negative_variance else var) ** 0.5
            density = np.minimum(1.0 / rms, (1.0 / np.sqrt(2.0 * np.pi)) * np.exp(-0.5 * ((obs - mean) / rms)) / rms)
            return dim_factor / density * rho

        with np.errstate(divide='ignore', invalid='ignore', over='ignore'):
            tbw = bandwidth(self.tmom1_gpu.get(), self.tmom2_gpu.get(), event_time, True)
            inv_tbw = np.zeros_like(tbw)
            inv_tbw[tbw > 0] = tbw[tbw > 0] ** -1
            self.inv_time_bandwidths_gpu = ga.to_gpu(inv_tbw.astype(np.float32))
            if self.time_only:
                self.inv_charge_bandwidths_gpu = ga.zeros(len(inv_tbw), np.float32)
            else:
                qbw = bandwidth(self.qmom1_gpu.get(), self.qmom2_gpu.get(), event_charge, False)
                self.inv_charge_bandwidths_gpu = ga.to_gpu((qbw ** -1).astype(np.float32))

    def setup_kernel(self, event_hit, event_time, event_charge):
        """pdf.py:114-132"""
        self.event_hit_gpu = ga.to_gpu(np.asarray(event_hit).astype(np.uint32))
        self.event_time_gpu = ga.to_gpu(np.asarray(event_time).astype(np.float32))
        self.event_charge_gpu = ga.to_gpu(np.asarray(event_charge).astype(np.float32))
        self.hitcount_gpu.fill(0)
        self.time_pdf_values_gpu = ga.zeros(len(event_hit), np.float32)
        self.charge_pdf_values_gpu = ga.zeros(len(event_hit), np.float32)

    def clear_kernel(self):
        self.hitcount_gpu.fill(0)
        self.time_pdf_values_gpu.fill(0)
        self.charge_pdf_values_gpu.fill(0)

    def accumulate_kernel(self, gpuchannels, nthreads_per_block=64):
        """pdf.py:139-158 -> accumulate_kernel_eval (pdf.cu:271-368)."""
        n = len(self.event_hit_gpu)
        if len(self.hitcount_gpu) < n:
            raise ValueError('setup_moments covered %d channels, the event has %d' % (len(self.hitcount_gpu), n))
        t, q = _channel_words(gpuchannels, n)
        _native.call('chr_pdf_accumulate_kernel_eval', int(bool(self.time_only)), n, self.event_hit_gpu.gpudata,
                     self.event_time_gpu.gpudata, self.event_charge_gpu.gpudata, t, q, _f(self.trange[0]),
                     _f(self.trange[1]), _f(self.qrange[0]), _f(self.qrange[1]),
                     self.inv_time_bandwidths_gpu.gpudata, self.inv_charge_bandwidths_gpu.gpudata,
                     self.hitcount_gpu.gpudata, self.time_pdf_values_gpu.gpudata,
                     self.charge_pdf_values_gpu.gpudata, current_stream())

    def get_kernel_eval(self):
        """pdf.py:161-175 -> (hitcount, pdf values, zero uncertainties).

        As in the reference, a channel whose charge bandwidth is NaN (its
        charge variance is not clipped at zero in compute_bandwidth,
        pdf.py:99-110) yields a NaN value when time and charge are combined."""
        hitcount = self.hitcount_gpu.get()
        norm = np.maximum(1, hitcount)
        time_pdf = self.time_pdf_values_gpu.get() / norm
        charge_pdf = self.charge_pdf_values_gpu.get() / norm
        values = time_pdf if self.time_only else time_pdf * charge_pdf
        return hitcount, values, np.zeros_like(values)


class GPUPDF(object):
    """Histogram PDFs and the adaptive-bin evaluation (pdf.py:177-372)."""

    def setup_pdf(self, nchannels, tbins, trange, qbins, qrange):
        """pdf.py:183-199: [channel, time bin, charge bin] u32 histogram."""
        self.events_in_histogram = 0
        self.hitcount_gpu = ga.zeros(nchannels, np.uint32)
        self.pdf_gpu = ga.zeros((nchannels, tbins, qbins), np.uint32)
        self.tbins, self.trange, self.qbins, self.qrange = tbins, trange, qbins, qrange

    def clear_pdf(self):
        self.hitcount_gpu.fill(0)
        self.pdf_gpu.fill(0)

    def add_hits_to_pdf(self, gpuchannels, nthreads_per_block=64):
        """pdf.py:206-222 -> bin_hits (pdf.cu:9-32)."""
        n = len(self.hitcount_gpu)
        t, q = _channel_words(gpuchannels, n)
        _native.call('chr_pdf_bin_hits', n, q, t, self.hitcount_gpu.gpudata, int(self.tbins), _f(self.trange[0]),
                     _f(self.trange[1]), int(self.qbins), _f(self.qrange[0]), _f(self.qrange[1]),
                     self.pdf_gpu.gpudata, current_stream())
        self.events_in_histogram += 1

    def get_pdfs(self):
        """(hitcount[nchannels], pdf[nchannels, tbins, qbins])"""
        return self.hitcount_gpu.get(), self.pdf_gpu.get().reshape(-1, self.tbins, self.qbins)

    def setup_pdf_eval(self, event_hit, event_time, event_charge, min_twidth, trange, min_qwidth, qrange,
                       min_bin_content=10, time_only=True):
        """pdf.py:229-287: evaluate the PDF at one event, bins widened until
        they hold min_bin_content MC entries (time only, as the reference)."""
        event_hit = np.asarray(event_hit)
        self.event_nhit = int(np.count_nonzero(event_hit))
        self.map_hit_offset_to_channel_id = np.where(event_hit)[0].astype(np.uint32)
        self.map_hit_offset_to_channel_id_gpu = ga.to_gpu(self.map_hit_offset_to_channel_id)
        self.map_channel_id_to_hit_offset = np.maximum(0, event_hit.cumsum() - 1).astype(np.uint32)
        self.map_channel_id_to_hit_offset_gpu = ga.to_gpu(self.map_channel_id_to_hit_offset)
        self.event_hit_gpu = ga.to_gpu(event_hit.astype(np.uint32))
        self.event_time_gpu = ga.to_gpu(np.asarray(event_time).astype(np.float32))
        self.event_charge_gpu = ga.to_gpu(np.asarray(event_charge).astype(np.float32))
        self.eval_hitcount_gpu = ga.zeros(len(event_hit), np.uint32)
        self.eval_bincount_gpu = ga.zeros(len(event_hit), np.uint32)
        self.nearest_mc_gpu = ga.empty(max(1, self.event_nhit * min_bin_content), np.float32)
        self.nearest_mc_gpu.fill(1e9)
        self.min_twidth, self.trange, self.min_qwidth, self.qrange = min_twidth, trange, min_qwidth, qrange
        self.min_bin_content = min_bin_content
        assert time_only   # pdf.py:286: only the time PDF is supported
        self.time_only = time_only

    def clear_pdf_eval(self):
        self.eval_hitcount_gpu.fill(0)
        self.eval_bincount_gpu.fill(0)
        self.nearest_mc_gpu.fill(1e9)

    def accumulate_pdf_eval(self, gpuchannels, nthreads_per_block=64, max_blocks=10000):
        """pdf.py:296-328 -> accumulate_bincount + accumulate_nearest_neighbor_block."""
        n = len(self.event_hit_gpu)
        ndaq = int(getattr(gpuchannels, 'ndaq', 1))
        t, _ = _channel_words(gpuchannels, n * ndaq)
        self.work_queues = ga.empty(max(1, self.event_nhit * (ndaq + 1)), np.uint32)
        self.work_queues.fill(1)
        _native.call('chr_pdf_accumulate_bincount', n, ndaq, self.event_hit_gpu.gpudata, self.event_time_gpu.gpudata,
                     t, self.eval_hitcount_gpu.gpudata, self.eval_bincount_gpu.gpudata, _f(self.min_twidth),
                     _f(self.trange[0]), _f(self.trange[1]), int(self.min_bin_content),
                     self.map_channel_id_to_hit_offset_gpu.gpudata, self.work_queues.gpudata, current_stream())
        _native.call('chr_pdf_accumulate_nearest', self.event_nhit, ndaq,
                     self.map_hit_offset_to_channel_id_gpu.gpudata, self.work_queues.gpudata,
                     self.event_time_gpu.gpudata, t, self.nearest_mc_gpu.gpudata, int(self.min_bin_content),
                     current_stream())

    def get_pdf_eval(self):
        """pdf.py:330-372 -> (hitcount, pdf value, pdf uncertainty) per channel."""
        evhit = self.event_hit_gpu.get().astype(bool)
        hitcount = self.eval_hitcount_gpu.get()
        bincount = self.eval_bincount_gpu.get()
        k = self.min_bin_content
        value = np.zeros(len(hitcount), dtype=float)
        frac_uncert = np.zeros_like(value)
        # enough MC inside the minimum-width bin: counting estimate
        high = bincount >= k
        if high.any():
            value[high] = bincount[high].astype(float) / hitcount[high] / self.min_twidth
            frac_uncert[high] = 1.0 / np.sqrt(bincount[high])
        # otherwise: the bin widened to the k-th nearest MC time
        low = ~high & (hitcount > 0) & evhit
        nearest = np.full((len(hitcount), k), 1e9, dtype=np.float32)
        nearest[self.map_hit_offset_to_channel_id, :] = \
            self.nearest_mc_gpu.get()[:self.event_nhit * k].reshape(self.event_nhit, k)
        last = np.maximum(0, (nearest < 1e9).astype(int).sum(axis=1) - 1)
        distance = nearest[np.arange(len(last)), last]
        if low.any():
            value[low] = (last[low] + 1).astype(float) / hitcount[low] / distance[low] / 2.0
            frac_uncert[low] = 1.0 / np.sqrt(last[low] + 1)
        return hitcount, value, value * frac_uncert
