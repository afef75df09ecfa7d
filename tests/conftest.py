import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the loader's BVH cache (chroma.cache, default ~/.chroma) goes to a per-session temp dir
os.environ['CHROMA_CACHE_DIR'] = tempfile.mkdtemp(prefix='chroma_cache_test_')
for p in (os.path.join(ROOT, 'chroma-lite_amd'), os.path.join(ROOT, 'oracle')):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device); run with -m gpu')


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope='session')
def small_detector():
    """2-PMT demo detector (the parity geometry; bit-identical to the
    reference's demo.detector(600, 900, 1500), see test_geometry_build)."""
    from chroma import demo, loader
    return loader.create_geometry_from_obj(demo.detector(600.0, 900.0, 1500.0))


@pytest.fixture(scope='session')
def small_packed(small_detector):
    from chroma.gpu.packing import PackedGeometry
    return PackedGeometry(small_detector)


@pytest.fixture(scope='session')
def cube_geometry():
    from chroma import make, loader
    return loader.create_geometry_from_obj(make.cube(1000.0))
