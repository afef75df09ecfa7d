"""Benchmark detectors (drop-in for reference chroma/demo/__init__.py:19-67):
8-inch PMTs with light cones placed along a spherical spiral inside a black
sphere filled with water.

detector()  -> 10,055 PMTs, 58.96 M triangles (the "~60M-triangle" config)
detector(pmt_radius=23780, sphere_radius=24280) -> the 29,007-PMT variant
tiny()      -> 53 PMTs, 389,568 triangles
"""
from math import sin, cos, sqrt

import numpy as np

from chroma.make import sphere
from chroma.geometry import Solid
from chroma.detector import Detector
from chroma.transform import make_rotation_matrix, normalize
from chroma.demo.pmt import build_8inch_pmt_with_lc
from chroma.demo.optics import water, black_surface
from chroma.log import logger


def spherical_spiral(radius, spacing):
    """Points ~`spacing` apart along a spiral covering a sphere of `radius`."""
    dl = spacing / radius
    t = 0.0
    a = np.pi / dl
    while t < np.pi:
        yield np.array([sin(t) * sin(a * t), sin(t) * cos(a * t), cos(t)]) * radius
        t += dl / sqrt(1 + a ** 2 * sin(t) ** 2)


def detector(pmt_radius=14000.0, sphere_radius=14500.0, spiral_step=350.0):
    pmt = build_8inch_pmt_with_lc()
    geo = Detector(water)
    geo.add_solid(Solid(sphere(sphere_radius, nsteps=200), water, water, surface=black_surface,
                        color=0xBBFFFFFF))
    y_axis = np.array((0.0, 1.0, 0.0))
    for position in spherical_spiral(pmt_radius, spiral_step):
        direction = -normalize(position)
        # the PMT model faces +y; its front face sits at `position`
        rotation = make_rotation_matrix(np.arccos(np.dot(y_axis, direction)), np.cross(direction, y_axis))
        geo.add_pmt(pmt, rotation, position)
    time_rms, charge_mean, charge_rms = 1.5, 1.0, 0.1
    geo.set_time_dist_gaussian(time_rms, -5 * time_rms, 5 * time_rms)
    geo.set_charge_dist_gaussian(charge_mean, charge_rms, 0.0, charge_mean + 5 * charge_rms)
    logger.info('Demo detector: %d PMTs', geo.num_channels())
    return geo


def tiny():
    return detector(2000.0, 2500.0, 700.0)


def geometry_hashes(det):
    """Counts and MD5s of a flattened detector: vertices (float32 bytes),
    triangles, solid_id and solid_id_to_channel_index (as int64) -- the record
    tests/golden/make_golden_geometry.py writes from the reference's own build
    (reference_hashes.json 'demo_detector' / 'detector_29k'), so a benchmark
    geometry is checked against the reference's generator."""
    import hashlib

    def md5(a):
        return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()
    det.flatten()
    return {'channels': int(det.num_channels()), 'triangles': int(len(det.mesh.triangles)),
            'vertices': int(len(det.mesh.vertices)),
            'md5_vertices': md5(np.asarray(det.mesh.vertices, np.float32)),
            'md5_triangles': md5(np.asarray(det.mesh.triangles).astype(np.int64)),
            'md5_solid_id': md5(np.asarray(det.solid_id).astype(np.int64)),
            'md5_solid_id_to_channel_index': md5(np.asarray(det.solid_id_to_channel_index).astype(np.int64))}
