"""The device region profile (reference CHROMA_DEVICE_PROFILE, profile.h:9-37,
profiler.py:207-288) on the HIP path: the profile build computes exactly what
the oracle computes, and its counters are consistent -- every work-item's
regions partition its kernel time, so the region cycles of each kernel add up
to the kernel's own cycles exactly; intersect_mesh is node + triangle steps."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_device_profile_regions(tmp_path, small_detector, small_packed):
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no HIP device')
    out = str(tmp_path / 'prof')
    env = dict(os.environ)
    env.pop('CHROMA_AMD_LIB', None)
    r = subprocess.run([sys.executable, os.path.join(HERE, 'device_profile_child.py'), out], env=env,
                       timeout=300, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    info = json.load(open(out + '.json'))
    got = np.load(out + '.npz')
    assert info['library'] == 'libchroma_amd_prof.so' and info['enabled']

    # the profile build computes what the oracle computes
    from chroma.photon_source import isotropic
    photons = isotropic(30000, seed=21)
    host = oracle.HostPhotons(photons)
    st = oracle.rng_init(64 * 1024, seed=1)
    oracle.propagate(small_packed, host, st, 64 * 1024, 64, 1024, 1000)
    assert np.array_equal(got['flags'], host.flags)
    assert np.array_equal(got['last_hit'], host.last_hit_triangles)
    assert np.allclose(got['pos'], host.pos, rtol=1e-5, atol=1e-5)
    assert np.array_equal(got['rng'], st)

    g = info['regions']
    c = {k: v['calls'] for k, v in g.items()}
    y = {k: v['cycles'] for k, v in g.items()}
    assert info['trace_launches'] > 0 and info['tail_photons'] > 0, info
    # walks: one per queued live ray of the trace launches (no flat walks here)
    assert 0 < c['intersect_mesh'] <= info['trace_rays']
    assert c['intersect_node'] >= c['intersect_mesh'] and c['intersect_triangle'] > 0
    assert c['intersect_box'] >= c['intersect_node']
    assert y['intersect_mesh'] == y['intersect_node'] + y['intersect_triangle']
    assert y['trace_kernel'] == (y['intersect_node'] + y['intersect_triangle'] + y['trace_refill']
                                 + y['trace_idle'] + y['trace_drain'])
    # every walk is either finished by its lane or handed to its draining wave
    assert c['trace_drain'] <= c['intersect_mesh']
    assert 0 < c['shade_physics'] <= c['fill_material']
    assert y['shade_kernel'] == y['fill_material'] + y['shade_physics'] + y['shade_other']
    assert c['tail_walk'] > 0 and c['tail_physics'] == c['tail_walk']
    assert y['tail_kernel'] == y['tail_walk'] + y['tail_physics'] + y['tail_other']
    assert c['fill_analytic'] == 0 and y['fill_analytic'] == 0
    for k in ('trace_kernel', 'shade_kernel', 'tail_kernel'):
        assert c[k] > 0 and y[k] > 0, k
    assert info['clock_khz'] > 0
    assert 'intersect_node' in info['report']
    # host side: the propagate call timed through chroma.gpu._native.call
    assert info['host']['chr_propagate']['calls'] == 1
    assert info['host']['chr_propagate']['total_ms'] > 0
