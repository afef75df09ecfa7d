#!/usr/bin/env python
"""Hashes of the benchmark geometries as the REFERENCE builds them (run ONLY in
the build container, where the read-only reference checkout exists at
/root/reference).

Imports the reference's pure-Python layer (chroma.demo, chroma.geometry,
chroma.detector), builds

  demo         chroma.demo.detector()                                  (C3)
  29k          chroma.demo.detector(pmt_radius=23780, sphere_radius=24280)
                                                               (headline bench)

flattens each with the reference's Geometry.flatten (geometry.py:337-391,
detector.py:134-140) and records MD5s of the vertices (float32 bytes), the
triangles (as int64), solid_id (as int64) and solid_id_to_channel_index (as
int64), plus counts, under the keys 'demo_detector' / 'detector_29k' of
tests/golden/reference_hashes.json.  Data only: no reference source travels.

    python tests/golden/make_golden_geometry.py [demo] [29k]

The 29k build holds ~20 GB of host memory at its peak (numpy's structured
np.unique over 85M vertex rows) and takes a few minutes.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference'

sys.path = [p for p in sys.path if 'chroma-lite_amd' not in p]
sys.path.insert(0, REF)

import chroma.demo as rdemo              # noqa: E402

BUILDS = {
    'demo': ('demo_detector', dict()),
    '29k': ('detector_29k', dict(pmt_radius=23780.0, sphere_radius=24280.0)),
}


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()


def geometry_hashes(det):
    """The record compared by chroma.demo.geometry_hashes (same fields)."""
    det.flatten()
    return {'channels': int(det.num_channels()), 'triangles': int(len(det.mesh.triangles)),
            'vertices': int(len(det.mesh.vertices)),
            'md5_vertices': md5(np.asarray(det.mesh.vertices, np.float32)),
            'md5_triangles': md5(np.asarray(det.mesh.triangles).astype(np.int64)),
            'md5_solid_id': md5(np.asarray(det.solid_id).astype(np.int64)),
            'md5_solid_id_to_channel_index': md5(np.asarray(det.solid_id_to_channel_index).astype(np.int64))}


def main(names):
    path = os.path.join(HERE, 'reference_hashes.json')
    with open(path) as f:
        hashes = json.load(f)
    for name in names:
        key, kw = BUILDS[name]
        t0 = time.time()
        rec = geometry_hashes(rdemo.detector(**kw))
        rec['params'] = kw
        rec['built_s'] = round(time.time() - t0, 1)
        hashes[key] = rec
        print(key, json.dumps(rec), flush=True)
        with open(path, 'w') as f:
            json.dump(hashes, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main(sys.argv[1:] or ['demo', '29k'])
