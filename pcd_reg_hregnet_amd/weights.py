"""Deterministic HRegNet weights for tests and the benchmark.

There is no trained registration-head checkpoint in the reference snapshot
(.MISSING_LARGE_BLOBS:2-4); the only trained weights are the feature
extractor's ``ckpt/pretrained/nusc_feats.pth`` (192 keys), kept as data under
``tests/golden/nusc_feats.npz``.  Heads (and, without that file, the feature
extractor) are filled by :func:`synthetic_value`, seeded per key name so the
values do not depend on module construction order or torch's RNG:

* conv weight / bias: U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (PyTorch's default bound)
* BN weight U(0.8, 1.2), bias N(0, 0.05), running_mean N(0, 0.1),
  running_var U(0.5, 1.5), num_batches_tracked 0
"""
from __future__ import annotations

import os
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
FEATS_NPZ = os.path.join(HERE, "..", "tests", "golden", "nusc_feats.npz")


def synthetic_value(name: str, shape, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
    shape = tuple(shape)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, np.int64)
    is_bn = len(shape) == 1 and leaf in ("weight", "bias", "running_mean", "running_var") and \
        not name.endswith(".0.bias")
    # conv biases live on index-0 modules of mlp heads ("mlp1.0.bias", "mlp3.0.bias")
    if leaf == "weight" and len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        b = 1.0 / np.sqrt(fan_in)
        return rng.uniform(-b, b, shape).astype(np.float32)
    if not is_bn:  # conv bias
        return rng.uniform(-0.05, 0.05, shape).astype(np.float32)
    if leaf == "weight":
        return rng.uniform(0.8, 1.2, shape).astype(np.float32)
    if leaf == "bias":
        return rng.normal(0.0, 0.05, shape).astype(np.float32)
    if leaf == "running_mean":
        return rng.normal(0.0, 0.1, shape).astype(np.float32)
    return rng.uniform(0.5, 1.5, shape).astype(np.float32)


def load_feats_npz(path: str = FEATS_NPZ) -> dict | None:
    if not os.path.exists(path):
        return None
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def make_state_dict(template: dict, seed: int = 0, pretrained_feats: bool = True) -> dict:
    """Fill every key of ``template`` (a state dict) deterministically.

    Keys under ``feature_extraction.`` come from nusc_feats.npz when present."""
    feats = load_feats_npz() if pretrained_feats else None
    out = {}
    for k, v in template.items():
        if feats is not None and k.startswith("feature_extraction."):
            arr = feats[k[len("feature_extraction."):]]
        else:
            arr = synthetic_value(k, v.shape, seed)
        out[k] = torch.from_numpy(np.array(arr)).to(v.dtype).reshape(v.shape)
    return out
