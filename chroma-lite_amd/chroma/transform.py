"""Rotation helpers (drop-in for reference chroma/transform.py)."""
import numpy as np


def norm(x):
    """Euclidean norm along the last axis."""
    return np.sqrt((x * x).sum(-1))


def normalize(x):
    """Unit vector(s) along x (float64)."""
    x = np.atleast_2d(np.asarray(x, dtype=float))
    return (x / norm(x)[:, np.newaxis]).squeeze()


def make_rotation_matrix(phi, n):
    """Matrix rotating points by phi counter-clockwise about axis n (looking
    towards +infinity): cos(phi) I + (1-cos(phi)) n n^T + sin(phi) [n]_x^T."""
    n = normalize(n)
    c, s = np.cos(phi), np.sin(phi)
    skew = np.array([[0, n[2], -n[1]], [-n[2], 0, n[0]], [n[1], -n[0], 0]])
    return c * np.identity(3) + (1 - c) * np.outer(n, n) + s * skew


def rotate(x, phi, n):
    """Rotate point(s) x by angle(s) phi about axis n (Rodrigues)."""
    n = normalize(n)
    x = np.atleast_2d(x)
    phi = np.atleast_1d(phi)
    c = np.cos(phi)[:, np.newaxis]
    s = np.sin(phi)[:, np.newaxis]
    return (x * c + n * np.dot(x, n)[:, np.newaxis] * (1 - c) + np.cross(x, n) * s).squeeze()


def rotate_matrix(x, phi, n):
    return np.inner(np.asarray(x), make_rotation_matrix(phi, n))


def get_perp(x):
    """An arbitrary vector perpendicular to x."""
    a = np.zeros(3)
    a[np.argmin(abs(x))] = 1
    return np.cross(a, x)


def gen_rot(a, b):
    """Matrix rotating vector a onto -b."""
    a = a / np.linalg.norm(a)
    b = b / np.linalg.norm(b)
    if (a == -b).all():
        return np.diag([1.0, 1.0, 1.0])
    if (a == b).all():
        v = np.cross(a, [0, 1, 0]) if (a[1] == 0 and a[2] == 0) else np.cross(a, [1, 0, 0])
        c = np.pi
    else:
        v = np.cross(a, b)
        c = np.arccos(-np.dot(a, b))
    return make_rotation_matrix(c, v)
