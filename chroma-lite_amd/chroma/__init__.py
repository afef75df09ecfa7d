"""chroma -- MI355X-native drop-in for youngsm/chroma-lite's optical photon
propagator.  Same import paths as the reference (chroma.sim.Simulation,
chroma.gpu.GPUPhotons, chroma.event, chroma.geometry, chroma.detector, ...);
the GPU path is hand-written HIP for gfx950 behind the C ABI in
include/chroma_amd.h (libchroma_amd.so), driven from here through ctypes.
"""
from chroma import geometry, detector, event, make, transform  # noqa: F401

__version__ = '0.1.0'
