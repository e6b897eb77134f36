"""Parameter inventory of the score network and a deterministic synthetic-weight generator.

The inventory mirrors the ``state_dict`` of the reference ``NCSN_LiDAR_small``
(LiDARGen/models/ncsnv2.py:420-482, blocks from LiDARGen/models/layers.py) key for key,
so a LiDARGen checkpoint loads without renaming.  No pretrained checkpoint exists
offline, so tests and benchmarks use ``synthetic_state_dict`` -- a name+shape keyed
PCG64 generator that gives the same tensors on every machine.
"""
from __future__ import annotations

import collections
import zlib

import numpy as np


def _conv(spec, name, cout, cin, k, bias=True):
    spec[name + ".weight"] = (cout, cin, k, k)
    if bias:
        spec[name + ".bias"] = (cout,)


def _norm(spec, name, c):
    # InstanceNorm2dPlus(bias=True): alpha, gamma, beta (normalization.py:150-161)
    spec[name + ".alpha"] = (c,)
    spec[name + ".gamma"] = (c,)
    spec[name + ".beta"] = (c,)


def _resblock(spec, name, cin, cout, down, dil):
    """ResidualBlock parameters (layers.py:401-441)."""
    if down:
        _conv(spec, name + ".conv1", cin, cin, 3)
        _norm(spec, name + ".normalize2", cin)
        if dil is None:  # ConvMeanPool conv2 and 1x1 ConvMeanPool shortcut
            _conv(spec, name + ".conv2.conv", cout, cin, 3)
            _conv(spec, name + ".shortcut.conv", cout, cin, 1)
        else:
            _conv(spec, name + ".conv2", cout, cin, 3)
            _conv(spec, name + ".shortcut", cout, cin, 3)
    else:
        _conv(spec, name + ".conv1", cout, cin, 3)
        _norm(spec, name + ".normalize2", cout)
        _conv(spec, name + ".conv2", cout, cout, 3)
        if cin != cout:
            _conv(spec, name + ".shortcut", cout, cin, 1)
    _norm(spec, name + ".normalize1", cin)


def _rcu(spec, name, c, n_blocks, n_stages=2):
    for i in range(n_blocks):
        for j in range(n_stages):
            _conv(spec, f"{name}.{i + 1}_{j + 1}_conv", c, c, 3, bias=False)


def _refine(spec, name, in_planes, features, start=False, end=False):
    """RefineBlock parameters (layers.py:214-232)."""
    for i, c in enumerate(in_planes):
        _rcu(spec, f"{name}.adapt_convs.{i}", c, 2)
    _rcu(spec, f"{name}.output_convs", features, 3 if end else 1)
    if not start:
        for i, c in enumerate(in_planes):
            _conv(spec, f"{name}.msf.convs.{i}", features, c, 3)
    for i in range(2):
        _conv(spec, f"{name}.crp.convs.{i}", features, features, 3, bias=False)


def param_spec(ngf: int = 128, channels: int = 2) -> "collections.OrderedDict[str, tuple]":
    """Every learnable tensor of NCSN_LiDAR_small (ncsnv2.py:420-482), name -> shape."""
    s: "collections.OrderedDict[str, tuple]" = collections.OrderedDict()
    _conv(s, "begin_conv", ngf, channels + 2, 3)
    _norm(s, "normalizer", ngf)
    _conv(s, "end_conv", channels, ngf, 3)
    _resblock(s, "res1.0", ngf, ngf, False, None)
    _resblock(s, "res1.1", ngf, ngf, False, None)
    _resblock(s, "res2.0", ngf, 2 * ngf, True, None)
    _resblock(s, "res2.1", 2 * ngf, 2 * ngf, False, None)
    _resblock(s, "res3.0", 2 * ngf, 2 * ngf, True, 2)
    _resblock(s, "res3.1", 2 * ngf, 2 * ngf, False, 2)
    _resblock(s, "res4.0", 2 * ngf, 2 * ngf, True, 4)
    _resblock(s, "res4.1", 2 * ngf, 2 * ngf, False, 4)
    _refine(s, "refine1", [2 * ngf], 2 * ngf, start=True)
    _refine(s, "refine2", [2 * ngf, 2 * ngf], 2 * ngf)
    _refine(s, "refine3", [2 * ngf, 2 * ngf], ngf)
    _refine(s, "refine4", [ngf, ngf], ngf, end=True)
    return s


def synthetic_param(key: str, shape: tuple) -> np.ndarray:
    """Deterministic float32 tensor for one parameter.

    Conv weights/biases are U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (PyTorch's default
    Conv2d bound); IN++ alpha/gamma are N(1, 0.02) as in normalization.py:156-158 and
    beta is N(0, 0.02) (non-zero so the bias path is exercised).
    """
    rng = np.random.Generator(np.random.PCG64(zlib.crc32(key.encode("utf-8"))))
    leaf = key.rsplit(".", 1)[-1]
    if leaf in ("alpha", "gamma"):
        v = 1.0 + 0.02 * rng.standard_normal(shape)
    elif leaf == "beta":
        v = 0.02 * rng.standard_normal(shape)
    elif leaf == "weight":
        fan_in = int(np.prod(shape[1:]))
        b = 1.0 / np.sqrt(fan_in)
        v = rng.uniform(-b, b, size=shape)
    elif leaf == "bias":
        v = rng.uniform(-0.05, 0.05, size=shape)
    else:
        raise KeyError(key)
    return v.astype(np.float32)


def get_sigmas_np(sigma_begin=50.0, sigma_end=0.01, num_classes=232, dist="geometric") -> np.ndarray:
    """models/__init__.py:5-18 get_sigmas, returned as the float32 numpy array the runners pass on."""
    if dist == "geometric":
        s = np.exp(np.linspace(np.log(sigma_begin), np.log(sigma_end), num_classes))
    elif dist == "uniform":
        s = np.linspace(sigma_begin, sigma_end, num_classes)
    else:
        raise NotImplementedError("sigma distribution not supported")
    return s.astype(np.float32)


def synthetic_state_dict(ngf: int = 128, channels: int = 2, num_classes: int = 232,
                         sigma_begin=50.0, sigma_end=0.01) -> "collections.OrderedDict[str, np.ndarray]":
    sd = collections.OrderedDict()
    sd["sigmas"] = get_sigmas_np(sigma_begin, sigma_end, num_classes)
    for k, shp in param_spec(ngf, channels).items():
        sd[k] = synthetic_param(k, shp)
    return sd
