"""Fixture (de)serialisation helpers shared by the golden generator and the tests.

A tensor is stored as float64 checksums (sum, sum|x|, sum x^2) in the JSON meta and
``SAMPLES`` values at fixed pseudo-random flat indices in the npz, so fixtures stay small
while still pinning every region of the tensor.
"""
import numpy as np
import torch

SAMPLES = 4096
PSAMPLES = 32


def _idx(n, k, salt):
    rng = np.random.default_rng([12345, n, salt])
    return np.sort(rng.choice(n, size=min(n, k), replace=False))


def summarize(arrays, meta, name, t, k=SAMPLES):
    a = t.detach().double().cpu().reshape(-1).numpy()
    meta[name] = {"shape": list(t.shape), "sum": float(a.sum()), "abs": float(np.abs(a).sum()),
                  "sq": float((a * a).sum())}
    arrays[name + "_samples"] = a[_idx(a.size, k, 0)].astype(np.float32)


def param_summary(arrays, meta, name, tensors):
    meta[name] = {}
    for key, t in tensors.items():
        if t is None:
            meta[name][key] = None
            continue
        a = t.detach().double().cpu().reshape(-1).numpy()
        meta[name][key] = {"norm": float(np.sqrt((a * a).sum())), "sum": float(a.sum())}
        arrays[name + ":" + key] = a[_idx(a.size, PSAMPLES, 1)].astype(np.float32)


def samples_of(t, k=SAMPLES, salt=0):
    a = t.detach().double().cpu().reshape(-1).numpy()
    return a[_idx(a.size, k, salt)]


def check_tensor(arrays, meta, name, t, rtol, atol=0.0):
    """Compare tensor ``t`` with the stored summary; returns max abs sample error."""
    m = meta[name]
    assert list(t.shape) == m["shape"], (name, list(t.shape), m["shape"])
    got = samples_of(t)
    ref = arrays[name + "_samples"].astype(np.float64)
    err = np.abs(got - ref)
    scale = np.abs(ref).max() + 1e-12
    assert (err <= atol + rtol * scale).all(), (name, float(err.max()), scale)
    a = t.detach().double().cpu().reshape(-1)
    assert abs(float(a.abs().sum()) - m["abs"]) <= rtol * m["abs"] + atol * a.numel(), name
    return float(err.max())


def check_params(arrays, meta, name, tensors, rtol, atol=0.0):
    """Every key of the fixture must be present in ``tensors`` and vice versa (a renamed or
    dropped parameter fails); a fixture entry of None (the reference produced no gradient)
    requires None or an all-zero tensor."""
    missing = sorted(set(meta[name]) ^ set(tensors))
    assert not missing, (name, "key sets differ", missing[:8])
    for key, t in tensors.items():
        m = meta[name][key]
        if m is None:
            assert t is None or float(t.detach().abs().max()) == 0.0, (name, key, "expected no gradient")
            continue
        got = samples_of(t, PSAMPLES, 1)
        ref = arrays[name + ":" + key].astype(np.float64)
        scale = max(np.abs(ref).max(), 1e-12)
        err = np.abs(got - ref).max()
        assert err <= atol + rtol * scale, (name, key, float(err), scale)
        a = t.detach().double().cpu().reshape(-1).numpy()
        norm = float(np.sqrt((a * a).sum()))
        assert abs(norm - m["norm"]) <= rtol * m["norm"] + atol, (name, key, norm, m["norm"])
