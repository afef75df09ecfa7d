"""Diagnose a switch that changes photons: run the test_switches_identical
workload (small detector, 4 batches, 64 x 256 slots) under several env
settings (each in a child process) and the oracle, and report which photons
differ from the oracle in each.  usage: diag_switch.py NAME=ENV:V,ENV:V ..."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ('pos', 'dir', 'pol', 'wavelengths', 't', 'flags', 'last_hit_triangles')


def _small():
    from chroma import demo, loader
    return loader.create_geometry_from_obj(demo.detector(600.0, 900.0, 1500.0))


def child(out, batched):
    sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'chroma-lite_amd')]
    from chroma import gpu
    from chroma.photon_source import isotropic
    det = gpu.GPUDetector(_small())
    sources = [isotropic(n, seed=29 + i) for i, n in enumerate([30000, 70000, 5000, 120000])]
    rng = gpu.get_rng_states(64 * 256, seed=3)
    gps = [gpu.GPUPhotons(s, copy_flags=True, copy_triangles=False, copy_weights=False) for s in sources]
    if batched:
        gpu.propagate_batches(gps, det, rng, nthreads_per_block=64, max_blocks=256, max_steps=1000)
    else:
        for gp in gps:
            gp.propagate(det, rng, nthreads_per_block=64, max_blocks=256, max_steps=1000)
    got = [gp.get() for gp in gps]
    np.savez(out, **{'%s_%d' % (f, i): getattr(g, f) for i, g in enumerate(got) for f in FIELDS})


def main():
    if sys.argv[1] == '--child':
        return child(sys.argv[2], sys.argv[3] == '1')
    sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'chroma-lite_amd')]
    import oracle
    from chroma.gpu.packing import PackedGeometry
    from chroma.photon_source import isotropic
    geo = _small()
    packed = PackedGeometry(geo)
    sources = [isotropic(n, seed=29 + i) for i, n in enumerate([30000, 70000, 5000, 120000])]
    states = oracle.rng_init(64 * 256, seed=3)
    hosts = []
    for s in sources:
        h = oracle.HostPhotons(s)
        h.last_hit_triangles[:] = -1
        h.weights[:] = 1
        oracle.propagate(packed, h, states, 64 * 256, 64, 256, 1000)
        hosts.append(h)
    for spec in sys.argv[1:]:
        name, _, envs = spec.partition('=')
        env = dict(os.environ)
        for kv in filter(None, envs.split(',')):
            k, v = kv.split(':')
            env[k] = v
        for batched in (0, 1):
            out = '/tmp/diag_%s_%d.npz' % (name, batched)
            subprocess.run([sys.executable, __file__, '--child', out, str(batched)], env=env, check=True, timeout=300)
            d = np.load(out)
            rep = {'config': name, 'batched': batched}
            for i, h in enumerate(hosts):
                bad = np.zeros(len(h.flags), bool)
                for f in FIELDS:
                    a, b = d['%s_%d' % (f, i)], getattr(h, f)
                    if f in ('flags', 'last_hit_triangles'):
                        diff = a != b
                    else:
                        diff = ~np.isclose(a.astype(np.float64), b.astype(np.float64), rtol=1e-5, atol=1e-5)
                    if diff.ndim > 1:
                        diff = diff.any(axis=1)
                    bad |= diff
                idx = np.flatnonzero(bad)
                rep['batch%d' % i] = {'n_diff': int(len(idx)), 'first': idx[:5].tolist(),
                                      'flags_gpu': d['flags_%d' % i][idx[:5]].tolist(),
                                      'flags_oracle': h.flags[idx[:5]].tolist(),
                                      'lht_gpu': d['last_hit_triangles_%d' % i][idx[:5]].tolist(),
                                      'lht_oracle': h.last_hit_triangles[idx[:5]].tolist()}
            print(json.dumps(rep), flush=True)


if __name__ == '__main__':
    main()
