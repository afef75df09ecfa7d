"""Device layer (drop-in for reference chroma/gpu/): GPUPhotons, GPUGeometry,
GPUDetector, RNG states, context helpers.  Everything launches hand-written
gfx950 HIP kernels through libchroma_amd.so (chroma.gpu._native)."""
from chroma.gpu.tools import (chunk_iterator, to_float3, to_uint3, create_cuda_context, get_rng_states,  # noqa
                              RNGStates, current_stream)
from chroma.gpu.geometry import GPUGeometry  # noqa: F401
from chroma.gpu.detector import GPUDetector  # noqa: F401
from chroma.gpu.photon import GPUPhotons, GPUPhotonsSlice, propagate_batches  # noqa: F401
from chroma.gpu.daq import GPUDaq, GPUChannels  # noqa: F401
from chroma.gpu.pdf import GPUPDF, GPUKernelPDF  # noqa: F401
from chroma.gpu.render import GPURays  # noqa: F401
