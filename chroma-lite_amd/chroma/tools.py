"""Small numeric helpers (drop-in for the parts of reference chroma/tools.py the
geometry builders and tests use)."""
import time

import numpy as np

from chroma.transform import normalize

try:  # line_profiler's builtin when running under kernprof
    profile_if_possible = profile  # noqa: F821
except NameError:
    def profile_if_possible(fn):
        return fn


def filled_array(value, shape, dtype):
    return np.full(shape, value, dtype=dtype)


def count_nonzero(array):
    return int((array != 0).sum())


def timeit(func):
    def wrapped(*args, **kwargs):
        t0 = time.time()
        out = func(*args, **kwargs)
        print('%s elapsed %1.2f sec' % (func.__name__, time.time() - t0))
        return out
    return wrapped


def read_csv(filename):
    """Rows of comma-separated floats; non-numeric lines are skipped."""
    rows = []
    with open(filename) as f:
        for line in f:
            try:
                rows.append([float(s) for s in line.split(',')])
            except ValueError:
                pass
    return np.array(rows)


def offset(points, x, tol=1e-9):
    """Offset the polyline `points` (2-D) sideways by distance x (positive:
    the path direction rotated 90 degrees clockwise).  Each new vertex is the
    intersection of the two neighbouring offset segments."""
    points = np.asarray(points)
    keep = np.ones(len(points), dtype=bool)
    keep[1:] = np.linalg.norm(points[1:] - points[:-1], axis=1) > tol
    points = points[keep]
    # mirror one extra point at each end so the end vertices have two segments
    ext = np.array([points[0] - (points[1] - points[0])] + list(points)
                   + [points[-1] - (points[-2] - points[-1])])

    def shifted(p, q):
        d = q - p
        n = np.array([d[1], -d[0]])         # (d, 0) x z-hat, exactly
        n /= np.linalg.norm(n)
        n *= x
        return p + n, q + n

    out = []
    for i in range(1, len(ext) - 1):
        a, b = shifted(ext[i - 1], ext[i])
        c, d = shifted(ext[i], ext[i + 1])
        m = np.empty((2, 2))
        m[:, 0] = b - a
        m[:, 1] = c - d
        try:
            j = np.linalg.solve(m, c - a)[0]
        except np.linalg.LinAlgError:
            out.append(b)
            continue
        out.append(a + j * (b - a))
    return np.array(out)


def from_film(position=(0, 0, 0), axis1=(0, 0, 1), axis2=(1, 0, 0), size=(800, 600), width=35.0,
              focal_length=18.0):
    """Rays from a pinhole camera: (positions, unit directions), one per pixel
    of a size[0] x size[1] film (reference tools.py:207-240)."""
    height = width * (size[1] / float(size[0]))
    axis1 = normalize(axis1)
    axis2 = normalize(axis2)
    dx0 = width / size[0]
    dx1 = height / size[1]
    yy, xx = np.meshgrid(np.arange(size[1]), np.arange(size[0]))
    n = size[0] * size[1]
    grid = -np.tile(axis2, (n, 1)) * xx.ravel()[:, np.newaxis] * dx0 + \
        np.tile(axis1, (n, 1)) * yy.ravel()[:, np.newaxis] * dx1
    grid += axis2 * width / 2 - axis1 * height / 2
    grid -= np.cross(axis1, axis2) * focal_length
    return np.tile(position, (n, 1)), normalize(-grid)
