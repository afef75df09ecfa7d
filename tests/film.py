"""Camera rays of the reference's ray-intersection KAT
(test/test_ray_intersection.py + data/ray_intersection.npy): one ray per pixel
of an 800x600 film, STARTING ON THE FILM (the layout the golden distances were
made with: the centre pixel reads 518 = 500 + focal length) and pointing
through the pinhole at the cube centre."""
import numpy as np


def film_rays(size=(800, 600), width=35.0, focal_length=18.0):
    a1 = np.array([0.0, 0.0, 1.0])
    a2 = np.array([1.0, 0.0, 0.0])
    height = width * (size[1] / float(size[0]))
    yy, xx = np.meshgrid(np.arange(size[1]), np.arange(size[0]))
    grid = (-a2[None, :] * xx.ravel()[:, None] * (width / size[0])
            + a1[None, :] * yy.ravel()[:, None] * (height / size[1]))
    grid += a2 * width / 2 - a1 * height / 2
    grid -= np.cross(a1, a2) * focal_length
    d = -grid
    d /= np.linalg.norm(d, axis=1)[:, None]
    return grid, d
