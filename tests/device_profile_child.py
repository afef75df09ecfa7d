"""Child process of tests/test_gpu_device_profile.py: loads the device-profile
build (CHROMA_DEVICE_PROFILE=1 must be set before the first native call, so it
runs in its own process), propagates a batch on the 2-PMT detector with the
split step kernels and the tail kernel, and writes the photons, the region
counters and the host profile.  usage: device_profile_child.py OUT_PREFIX"""
import json
import os
import sys

os.environ['CHROMA_DEVICE_PROFILE'] = '1'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'chroma-lite_amd'))

import numpy as np  # noqa: E402


def main(out):
    import torch
    from chroma import demo, gpu, loader
    from chroma.gpu import _native, profiler
    from chroma.photon_source import isotropic
    torch.cuda.set_device(0)
    geo = loader.create_geometry_from_obj(demo.detector(600.0, 900.0, 1500.0))
    photons = isotropic(30000, seed=21)
    gg = gpu.GPUGeometry(geo)
    gp = gpu.GPUPhotons(photons)
    rng = gpu.get_rng_states(64 * 1024, seed=1)
    profiler.enable()
    profiler.device_reset()
    gp.propagate(gg, rng, nthreads_per_block=64, max_blocks=1024, max_steps=1000)
    regions = profiler.device_fetch()
    text = profiler.device_report()
    got = gp.get()
    np.savez(out + '.npz', flags=got.flags, last_hit=got.last_hit_triangles, pos=got.pos, dir=got.dir,
             t=got.t, rng=rng.get().reshape(-1))
    st = gp.last_stats
    json.dump({'library': os.path.basename(_native.library_path()),
               'enabled': profiler.device_available(), 'regions': regions,
               'clock_khz': profiler.device_fetch.clock_khz, 'report': text, 'host': profiler.stats(),
               'trace_rays': int(st.trace_rays), 'trace_launches': int(st.trace_launches),
               'tail_photons': int(st.tail_photons), 'steps_run': int(st.steps_run)},
              open(out + '.json', 'w'), indent=1)


if __name__ == '__main__':
    main(sys.argv[1])
