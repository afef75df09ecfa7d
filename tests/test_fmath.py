"""The portable math of include/chroma_fmath.h against float64 numpy."""
import numpy as np

import oracle


def ulp_err(got, exact):
    got = got.astype(np.float64)
    spacing = np.spacing(np.abs(exact).astype(np.float32)).astype(np.float64)
    return np.abs(got - exact) / spacing


def test_log_exp():
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(1e-10, 1, 20000), rng.uniform(1, 1e6, 20000),
                        (np.arange(1, 2 ** 16, 7, dtype=np.float64) * 2.0 ** -32)]).astype(np.float32)
    assert ulp_err(oracle.math('log', x), np.log(x.astype(np.float64))).max() <= 2
    y = rng.uniform(-80, 80, 40000).astype(np.float32)
    assert ulp_err(oracle.math('exp', y), np.exp(y.astype(np.float64))).max() <= 2


def test_trig():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-7, 7, 40000), rng.uniform(-200, 200, 10000)]).astype(np.float32)
    x64 = x.astype(np.float64)
    for name, fn in (('sin', np.sin), ('cos', np.cos)):
        err = np.abs(oracle.math(name, x).astype(np.float64) - fn(x64))
        assert err.max() < 2e-7
    t = rng.uniform(-1.5, 1.5, 20000).astype(np.float32)
    assert ulp_err(oracle.math('tan', t), np.tan(t.astype(np.float64))).max() <= 4


def test_inverse_trig():
    rng = np.random.default_rng(2)
    x = np.concatenate([rng.uniform(-1, 1, 40000), [-1, 1, 0, 0.5, -0.5]]).astype(np.float32)
    x64 = x.astype(np.float64)
    assert np.abs(oracle.math('asin', x) - np.arcsin(x64)).max() < 3e-7
    assert np.abs(oracle.math('acos', x) - np.arccos(x64)).max() < 5e-7
    assert np.isnan(oracle.math('acos', np.array([1.5], np.float32))).all()
    y = rng.normal(size=20000).astype(np.float32)
    z = rng.normal(size=20000).astype(np.float32)
    assert np.abs(oracle.math('atan2', z, y) - np.arctan2(y.astype(np.float64), z.astype(np.float64))).max() < 5e-7
