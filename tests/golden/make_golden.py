#!/usr/bin/env python
"""Golden-fixture generator (run ONLY in the build container, where the
read-only reference checkout exists at /root/reference).

It imports the reference's *pure-Python* layer (chroma.geometry, chroma.demo,
chroma.detector, chroma.make, chroma.stl, chroma.models -- the CUDA/PyCUDA
parts are absent in this container) and writes small,
data-only fixtures into tests/golden/ and package data into
chroma-lite_amd/chroma/demo/data/:

  optics.npz          raw (wavelength, value) tables of the demo materials and
                      surfaces (reference chroma/demo/optics.py)
  pmt_profiles.npz    the PMT / light-cone profile point lists (reference
                      chroma/demo/sno_pmt.txt, sno_cone.txt)
  pmt_lc_solid.npz    the 8" PMT + light-cone solid as the reference builds it
                      (chroma/demo/pmt.py:build_8inch_pmt_with_lc)
  detector_small.npz  a flattened 2-PMT demo detector (geometry.py:337-391,
                      detector.py:134-140) used as the parity geometry
  lionsolid.npz       the lionsolid mesh (chroma/models) for config C1
  ray_intersection.npy copied data file of the reference test suite
                      (test/data/ray_intersection.npy)
  cube_1000.npz       chroma.make.cube(1000) mesh (test_ray_intersection.py)
  reference_hashes.json  counts/MD5s of larger reference objects (demo.tiny())

No reference source text is copied; only numeric data produced by running it.
"""
import hashlib
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, '..', '..'))
PKGDATA = os.path.join(REPO, 'chroma-lite_amd', 'chroma', 'demo', 'data')
REF = '/root/reference'

sys.path = [p for p in sys.path if 'chroma-lite_amd' not in p]
sys.path.insert(0, REF)

import chroma.geometry as rgeo          # noqa: E402
import chroma.demo as rdemo              # noqa: E402
import chroma.demo.optics as roptics     # noqa: E402
import chroma.make as rmake              # noqa: E402
import chroma.tools as rtools            # noqa: E402


def md5(*arrays):
    h = hashlib.md5()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def export_optics():
    out = {}
    mats = {'water': roptics.water, 'glass': roptics.glass, 'vacuum': roptics.vacuum}
    for name, m in mats.items():
        for prop in ('refractive_index', 'absorption_length', 'scattering_length'):
            out['material/%s/%s' % (name, prop)] = np.asarray(getattr(m, prop), dtype=np.float64)
    surfs = {'black_surface': roptics.black_surface, 'shiny_surface': roptics.shiny_surface,
             'r7081hqe_photocathode': roptics.r7081hqe_photocathode,
             'lambertian_surface': roptics.lambertian_surface,
             'glossy_surface': roptics.glossy_surface}
    for name, s in surfs.items():
        for prop in ('detect', 'absorb', 'reemit', 'reflect_diffuse', 'reflect_specular',
                     'eta', 'k', 'reemission_cdf'):
            out['surface/%s/%s' % (name, prop)] = np.asarray(getattr(s, prop), dtype=np.float64)
    os.makedirs(PKGDATA, exist_ok=True)
    np.savez_compressed(os.path.join(PKGDATA, 'optics.npz'), **out)


def export_profiles():
    d = os.path.join(REF, 'chroma', 'demo')
    pmt = rtools.read_csv(os.path.join(d, 'sno_pmt.txt'))
    cone = rtools.read_csv(os.path.join(d, 'sno_cone.txt'))
    np.savez_compressed(os.path.join(PKGDATA, 'pmt_profiles.npz'), sno_pmt=pmt, sno_cone=cone)


def solid_arrays(solid, prefix=''):
    names = lambda objs: np.array([('' if o is None else o.name) for o in objs])
    return {prefix + 'vertices': solid.mesh.vertices, prefix + 'triangles': solid.mesh.triangles,
            prefix + 'material1': names(solid.material1), prefix + 'material2': names(solid.material2),
            prefix + 'surface': names(solid.surface), prefix + 'color': solid.color}


def export_pmt_solid():
    from chroma.demo.pmt import build_8inch_pmt_with_lc
    pmt = build_8inch_pmt_with_lc()
    np.savez_compressed(os.path.join(HERE, 'pmt_lc_solid.npz'), **solid_arrays(pmt))


def flat_detector_arrays(det):
    det.flatten()
    g = det
    mat_names = np.array([m.name for m in g.unique_materials])
    surf_names = np.array([('' if s is None else s.name) for s in g.unique_surfaces])
    return dict(vertices=g.mesh.vertices, triangles=g.mesh.triangles, solid_id=g.solid_id,
                material1_index=g.material1_index, material2_index=g.material2_index,
                surface_index=g.surface_index, colors=g.colors,
                material_names=mat_names, surface_names=surf_names,
                solid_id_to_channel_index=np.asarray(g.solid_id_to_channel_index),
                channel_index_to_solid_id=np.asarray(g.channel_index_to_solid_id),
                time_cdf_x=np.asarray(g.time_cdf[0]), time_cdf_y=np.asarray(g.time_cdf[1]),
                charge_cdf_x=np.asarray(g.charge_cdf[0]), charge_cdf_y=np.asarray(g.charge_cdf[1]),
                detector_material=np.array(g.detector_material.name))


def export_small_detector():
    # demo.detector() with radii chosen so the spiral places two PMTs
    det = rdemo.detector(pmt_radius=600.0, sphere_radius=900.0, spiral_step=1500.0)
    arrs = flat_detector_arrays(det)
    arrs['params'] = np.array([600.0, 900.0, 1500.0])
    np.savez_compressed(os.path.join(HERE, 'detector_small.npz'), **arrs)
    return int(det.num_channels()), len(arrs['triangles'])


def export_lionsolid():
    import chroma.models as models
    mesh = models.lionsolid()
    np.savez_compressed(os.path.join(HERE, 'lionsolid.npz'), vertices=mesh.vertices,
                        triangles=mesh.triangles)
    return len(mesh.triangles)


def export_cube_and_rays():
    shutil.copyfile(os.path.join(REF, 'test', 'data', 'ray_intersection.npy'),
                    os.path.join(HERE, 'ray_intersection.npy'))
    cube = rmake.cube(1000.0)
    np.savez_compressed(os.path.join(HERE, 'cube_1000.npz'), vertices=cube.vertices,
                        triangles=cube.triangles)
    pos, dir = rtools.from_film()
    return md5(np.asarray(pos, np.float64), np.asarray(dir, np.float64))


def main():
    export_optics()
    export_profiles()
    export_pmt_solid()
    hashes = {}
    nch, ntri = export_small_detector()
    hashes['detector_small'] = {'channels': nch, 'triangles': ntri}
    hashes['lionsolid_triangles'] = export_lionsolid()
    hashes['from_film_md5'] = export_cube_and_rays()
    sph = rmake.sphere(2500.0, nsteps=200)
    hashes['sphere_2500_200'] = {'vertices': len(sph.vertices), 'triangles': len(sph.triangles),
                                 'md5_triangles': md5(sph.triangles.astype(np.int64))}
    tiny = rdemo.tiny()
    a = flat_detector_arrays(tiny)
    hashes['tiny'] = {'channels': int(tiny.num_channels()), 'triangles': len(a['triangles']),
                      'vertices': len(a['vertices']),
                      'md5_triangles': md5(a['triangles'].astype(np.int64)),
                      'md5_solid_id': md5(a['solid_id'].astype(np.int64)),
                      'vertex_sum': float(np.asarray(a['vertices'], np.float64).sum()),
                      'vertex_abs_sum': float(np.abs(np.asarray(a['vertices'], np.float64)).sum())}
    with open(os.path.join(HERE, 'reference_hashes.json'), 'w') as f:
        json.dump(hashes, f, indent=1, sort_keys=True)
    print(json.dumps(hashes, indent=1))


if __name__ == '__main__':
    main()
