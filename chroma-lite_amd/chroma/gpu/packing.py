"""Flatten a Geometry into the plain arrays of chr_geometry_desc.

This mirrors what the reference GPUGeometry computes before uploading
(chroma/gpu/geometry.py:14-520): every material/surface property is linearly
interpolated onto one wavelength grid (np.interp, then float32), component
time CDFs onto one time grid, material codes packed as
m1<<24 | m2<<16 | surface<<8, materials/surfaces referenced only by analytic
wire planes appended after the mesh ones.  Each table gets one trailing pad
element (a copy of its last value): the reference's interp_property reads one
element past the table at the last grid point.
"""
import ctypes

import numpy as np

from chroma.geometry import standard_wavelengths
from chroma.gpu import _native


def _interp(grid, prop):
    assert prop is not None, 'property must not be None'
    prop = np.asarray(prop)
    return np.interp(grid, prop[:, 0], prop[:, 1]).astype(np.float32)


def _pad(a):
    a = np.asarray(a, dtype=np.float32)
    return np.ascontiguousarray(np.concatenate([a, a[-1:]]))


def _pad_rows(rows, n):
    if len(rows) == 0:
        return np.zeros((0, n + 1), dtype=np.float32)
    return np.ascontiguousarray(np.stack([_pad(r) for r in rows]))


def _uniform_step(grid, what):
    steps = np.unique(np.diff(grid))
    if len(steps) != 1:
        raise ValueError('%s must be equally spaced apart.' % what)
    return steps.item()


class PackedGeometry(object):
    """Host arrays for one geometry; .desc() returns the ctypes descriptor
    (valid while this object is alive)."""

    def __init__(self, geometry, wavelengths=None, times=None):
        wavelengths = standard_wavelengths if wavelengths is None else np.asarray(wavelengths)
        wstep = _uniform_step(wavelengths, 'wavelengths')
        if times is None:
            tstep = 0.05
            times = np.arange(0, 1000, tstep)
        else:
            tstep = _uniform_step(times, 'times')
        self.wavelengths, self.times = wavelengths, times
        self.wavelength_step, self.time_step = np.float32(wstep), np.float32(tstep)
        W, T = len(wavelengths), len(times)
        mesh = geometry.mesh
        bvh = getattr(geometry, 'bvh', None)
        if bvh is None:
            raise ValueError('geometry has no BVH: build one with chroma.loader.load_bvh / '
                             'chroma.bvh.make_recursive_grid_bvh')
        self.vertices = np.ascontiguousarray(mesh.vertices, dtype=np.float32)
        self.triangles = np.ascontiguousarray(mesh.triangles, dtype=np.uint32)
        self.nodes = np.ascontiguousarray(bvh.nodes).view(np.uint32).reshape(-1, 4)
        self.world_origin = np.asarray(bvh.world_coords.world_origin, dtype=np.float32)
        self.world_scale = np.float32(bvh.world_coords.world_scale)

        materials = list(geometry.unique_materials)
        surfaces = list(geometry.unique_surfaces)
        planes = list(getattr(geometry, 'wireplanes', None) or [])
        for desc in planes:     # materials/surfaces used only by wire planes (geometry.py:109-163, 265-339)
            for key in ('material_inner', 'material_outer'):
                m = desc.get(key) if isinstance(desc, dict) else getattr(desc, key, None)
                if m is not None and not any(m is x for x in materials):
                    materials.append(m)
            s = desc.get('surface') if isinstance(desc, dict) else getattr(desc, 'surface', None)
            if s is not None and not any(s is x for x in surfaces):
                surfaces.append(s)
        if len(materials) > 127 or len(surfaces) > 127:
            raise ValueError('at most 127 materials and 127 surfaces fit the 8-bit material codes')

        self.materials = []
        for m in materials:
            if m is None:
                raise Exception('one or more triangles is missing a material.')
            n = len(m.comp_reemission_prob)
            for name in ('comp_reemission_wvl_cdf', 'comp_reemission_time_cdf', 'comp_absorption_length'):
                assert len(getattr(m, name)) == n, 'component arrays must be same length'
            self.materials.append(dict(
                num_comp=n,
                refractive_index=_pad(_interp(wavelengths, m.refractive_index)),
                absorption_length=_pad(_interp(wavelengths, m.absorption_length)),
                scattering_length=_pad(_interp(wavelengths, m.scattering_length)),
                comp_reemission_prob=_pad_rows([_interp(wavelengths, c) for c in m.comp_reemission_prob], W),
                comp_reemission_wvl_cdf=_pad_rows([_interp(wavelengths, c) for c in m.comp_reemission_wvl_cdf], W),
                comp_reemission_time_cdf=_pad_rows([_interp(times, c) for c in m.comp_reemission_time_cdf], T),
                comp_absorption_length=_pad_rows([_interp(wavelengths, c) for c in m.comp_absorption_length], W)))
        self.surfaces = []
        for s in surfaces:
            if s is None:
                self.surfaces.append(None)
                continue
            d = dict(model=int(s.model), transmissive=int(s.transmissive), thickness=float(s.thickness))
            for name in ('detect', 'absorb', 'reemit', 'reflect_diffuse', 'reflect_specular', 'eta', 'k',
                         'reemission_cdf'):
                d[name] = _pad(_interp(wavelengths, getattr(s, name)))
            dp = getattr(s, 'dichroic_props', None)
            if dp:
                d['dichroic_angles'] = np.ascontiguousarray(dp.angles, dtype=np.float32)
                d['dichroic_reflect'] = _pad_rows([_interp(wavelengths, r) for r in dp.dichroic_reflect], W)
                d['dichroic_transmit'] = _pad_rows([_interp(wavelengths, r) for r in dp.dichroic_transmit], W)
            ap = getattr(s, 'angular_props', None)
            if ap:
                for name, arr in (('angular_angles', ap.angles), ('angular_transmit', ap.transmit),
                                  ('angular_reflect_specular', ap.reflect_specular),
                                  ('angular_reflect_diffuse', ap.reflect_diffuse)):
                    d[name] = np.ascontiguousarray(arr, dtype=np.float32)
            self.surfaces.append(d)

        self.material_codes = (((np.asarray(geometry.material1_index) & 0xff) << 24) |
                               ((np.asarray(geometry.material2_index) & 0xff) << 16) |
                               ((np.asarray(geometry.surface_index) & 0xff) << 8)).astype(np.uint32)

        self.wireplanes = []
        for desc in planes:
            get = (lambda k, default=None: desc.get(k, default)) if isinstance(desc, dict) else \
                (lambda k, default=None: getattr(desc, k, default))

            def index_of(objs, obj, direct):
                if direct is not None:
                    return int(direct)
                for i, x in enumerate(objs):
                    if x is obj:
                        return i
                return -1
            sidx = index_of(surfaces, get('surface'), get('surface_index'))
            mo = index_of(materials, get('material_outer'), get('material_outer_index'))
            mi = index_of(materials, get('material_inner'), get('material_inner_index'))
            if sidx < 0 or mo < 0 or mi < 0:
                raise ValueError('WirePlane surface/material unresolved')
            self.wireplanes.append(dict(
                origin=np.asarray(get('origin'), np.float32), u=np.asarray(get('u'), np.float32),
                v=np.asarray(get('v'), np.float32), pitch=float(np.float32(get('pitch'))),
                radius=float(np.float32(get('radius'))), umin=float(np.float32(get('umin', -1e9))),
                umax=float(np.float32(get('umax', 1e9))), vmin=float(np.float32(get('vmin', -1e9))),
                vmax=float(np.float32(get('vmax', 1e9))), v0=float(np.float32(get('v0', 0.0))),
                surface_index=sidx, material_outer_index=mo, material_inner_index=mi,
                color=int(get('color', 0))))
        self._desc = None

    def desc(self):
        """ctypes chr_geometry_desc pointing into this object's arrays."""
        if self._desc is not None:
            return self._desc
        ptr = lambda a: a.ctypes.data if a is not None and a.size else None   # noqa: E731
        mats = (_native.MaterialDesc * len(self.materials))()
        for i, m in enumerate(self.materials):
            mats[i] = _native.MaterialDesc(m['num_comp'], ptr(m['refractive_index']), ptr(m['absorption_length']),
                                           ptr(m['scattering_length']), ptr(m['comp_reemission_prob']),
                                           ptr(m['comp_reemission_wvl_cdf']), ptr(m['comp_reemission_time_cdf']),
                                           ptr(m['comp_absorption_length']))
        surfs = (_native.SurfaceDesc * max(1, len(self.surfaces)))()
        for i, s in enumerate(self.surfaces):
            if s is None:
                surfs[i] = _native.SurfaceDesc()
                continue
            sd = _native.SurfaceDesc()
            sd.present, sd.model, sd.transmissive, sd.thickness = 1, s['model'], s['transmissive'], s['thickness']
            for name in ('detect', 'absorb', 'reemit', 'reflect_diffuse', 'reflect_specular', 'eta', 'k',
                         'reemission_cdf'):
                setattr(sd, name, ptr(s[name]))
            if 'dichroic_angles' in s:
                sd.dichroic_nangles = len(s['dichroic_angles'])
                sd.dichroic_angles = ptr(s['dichroic_angles'])
                sd.dichroic_reflect = ptr(s['dichroic_reflect'])
                sd.dichroic_transmit = ptr(s['dichroic_transmit'])
            if 'angular_angles' in s:
                sd.angular_nangles = len(s['angular_angles'])
                for name in ('angular_angles', 'angular_transmit', 'angular_reflect_specular',
                             'angular_reflect_diffuse'):
                    setattr(sd, name, ptr(s[name]))
            surfs[i] = sd
        planes = (_native.WirePlaneDesc * max(1, len(self.wireplanes)))()
        for i, p in enumerate(self.wireplanes):
            wp = _native.WirePlaneDesc()
            wp.origin[:] = list(p['origin']); wp.u[:] = list(p['u']); wp.v[:] = list(p['v'])
            for k in ('pitch', 'radius', 'umin', 'umax', 'vmin', 'vmax', 'v0', 'surface_index',
                      'material_outer_index', 'material_inner_index', 'color'):
                setattr(wp, k, p[k])
            planes[i] = wp
        d = _native.GeometryDesc()
        d.nvertices, d.ntriangles, d.nnodes = len(self.vertices), len(self.triangles), len(self.nodes)
        d.nmaterials, d.nsurfaces, d.nwireplanes = len(self.materials), len(self.surfaces), len(self.wireplanes)
        d.h_vertices, d.h_triangles = ptr(self.vertices), ptr(self.triangles)
        d.h_material_codes, d.h_nodes = ptr(self.material_codes), ptr(self.nodes)
        d.world_origin[:] = [float(x) for x in self.world_origin]
        d.world_scale = float(self.world_scale)
        d.wavelength_n, d.wavelength_start, d.wavelength_step = len(self.wavelengths), float(self.wavelengths[0]), \
            float(self.wavelength_step)
        d.time_n, d.time_start, d.time_step = len(self.times), float(self.times[0]), float(self.time_step)
        d.materials = ctypes.cast(mats, ctypes.POINTER(_native.MaterialDesc))
        d.surfaces = ctypes.cast(surfs, ctypes.POINTER(_native.SurfaceDesc))
        d.wireplanes = ctypes.cast(planes, ctypes.POINTER(_native.WirePlaneDesc)) if self.wireplanes else None
        self._keep = (mats, surfs, planes)
        self._desc = d
        return d
