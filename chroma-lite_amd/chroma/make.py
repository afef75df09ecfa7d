"""Mesh primitives (drop-in for reference chroma/make.py).

Both extrusions build a (rows x columns) grid of vertex indices and stitch each
quad of neighbouring grid points into two triangles, wrapping around the
columns (reference make.py:6-93), so meshes come out vertex-for-vertex equal
to the reference's (tests/test_geometry_build.py checks cube and sphere).
"""
import numpy as np

from chroma.geometry import Mesh
from chroma.transform import rotate


def mesh_grid(grid):
    """Two triangles per grid cell: (a, b, b') and (a, b', a') where b is the
    next row and ' the next column (cyclic)."""
    grid = np.asarray(grid)
    a = grid[:-1].ravel()
    b = grid[1:].ravel()
    a_next = np.roll(grid[:-1], -1, 1).ravel()
    b_next = np.roll(grid[1:], -1, 1).ravel()
    first = np.stack((a, b, b_next), axis=1)
    second = np.stack((a, b_next, a_next), axis=1)
    return np.concatenate((first, second)).astype(grid.dtype)


def linear_extrude(x1, y1, height, x2=None, y2=None, center=None, endcaps=True):
    """Solid formed by extruding the counter-clockwise polygon (x1, y1) at
    z=-height/2 to (x2, y2) at z=+height/2 (tapered if x2/y2 differ)."""
    if len(x1) != len(y1):
        raise Exception('`x` and `y` arrays must have the same length.')
    x2 = x1 if x2 is None else x2
    y2 = y1 if y2 is None else y2
    if len(x2) != len(y2) or len(x2) != len(x1):
        raise Exception('`x` and `y` arrays must have the same length.')
    n = len(x1)
    lo, hi = -height / 2.0, height / 2.0
    rings = [np.column_stack((np.asarray(x1, float), np.asarray(y1, float), np.full(n, lo))),
             np.column_stack((np.asarray(x2, float), np.asarray(y2, float), np.full(n, hi)))]
    if endcaps:
        rings = ([np.column_stack((np.zeros(n), np.zeros(n), np.full(n, lo)))] + rings
                 + [np.column_stack((np.zeros(n), np.zeros(n), np.full(n, hi)))])
    k = len(rings)
    # vertex order: for each polygon point i, one vertex from every ring
    vertices = np.stack(rings, axis=1).reshape(n * k, 3)
    if center is not None:
        vertices = vertices + center
    grid = np.arange(n * k).reshape((n, k)).transpose()[::-1]
    return Mesh(vertices, mesh_grid(grid), remove_duplicate_vertices=True)


def rotate_extrude(x, y, nsteps=64):
    """Solid of revolution of the counter-clockwise profile (x, y) about the
    y axis, sampled at nsteps angles."""
    if len(x) != len(y):
        raise Exception('`x` and `y` arrays must have the same length.')
    points = np.array([x, y, np.zeros(len(x))]).transpose()
    angles = np.linspace(0, 2 * np.pi, nsteps, endpoint=False)
    vertices = np.vstack([rotate(points, a, (0, -1, 0)) for a in angles])
    grid = np.arange(len(vertices)).reshape((len(angles), len(points))).transpose()[::-1]
    return Mesh(vertices, mesh_grid(grid), remove_duplicate_vertices=True)


def box(dx, dy, dz, center=(0, 0, 0)):
    return linear_extrude([-dx / 2.0, dx / 2.0, dx / 2.0, -dx / 2.0],
                          [-dy / 2.0, -dy / 2.0, dy / 2.0, dy / 2.0], height=dz, center=center)


def cube(size, height=None, center=(0, 0, 0)):
    h = size / 2.0
    return linear_extrude([-h, h, h, -h], [-h, -h, h, h], height=size, center=center)


def cylinder_along_z(radius, height, points=100):
    angles = np.linspace(0, 2 * np.pi, points, endpoint=False)
    return linear_extrude(radius * np.cos(angles), radius * np.sin(angles), height)


def cylinder(radius, height, radius2=None, nsteps=64):
    radius2 = radius if radius2 is None else radius2
    return rotate_extrude([0, radius, radius2, 0], [-height / 2.0, -height / 2.0, height / 2.0, height / 2.0],
                          nsteps)


def segmented_cylinder(radius, height, nsteps=64, nsegments=100):
    nr = int((nsegments * radius / (2 * radius + height)) / 2)
    nh = int((nsegments * height / (2 * radius + height)) / 2)
    x = np.concatenate([np.linspace(0, radius, nr, endpoint=False), [radius] * nh,
                        np.linspace(radius, 0, nr, endpoint=False), [0]])
    y = np.concatenate([[-height / 2.0] * nr, np.linspace(-height / 2.0, height / 2.0, nh, endpoint=False),
                        [height / 2.0] * (nr + 1)])
    return rotate_extrude(x, y, nsteps)


def sphere(radius, nsteps=64):
    theta = np.linspace(-np.pi / 2, np.pi / 2, nsteps)
    return rotate_extrude(radius * np.cos(theta), radius * np.sin(theta), nsteps)


def torus(radius, offset, nsteps=64, circle_steps=None):
    circle_steps = nsteps if circle_steps is None else circle_steps
    a = np.linspace(0, 2 * np.pi, circle_steps)
    return rotate_extrude(radius * np.cos(a) + offset, radius * np.sin(a), nsteps)


def convex_polygon(x, y):
    vertices = np.column_stack((x, y, np.zeros_like(x)))
    n = len(vertices)
    triangles = np.column_stack((np.zeros(n - 2, np.int32), np.arange(1, n - 1), np.arange(2, n)))
    return Mesh(vertices=vertices, triangles=triangles)
