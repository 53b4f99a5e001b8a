"""Seeded synthetic weights with the reference's state_dict keys.

No trained checkpoint exists, so benchmarks and parity fixtures use
weights generated from (key, shape, seed) alone: He-normal conv weights
(std = sqrt(2 / fan_in)), BN gamma = 1, beta = 0, running stats 0 / 1, biases 0. Fixtures
additionally carry BN running statistics calibrated on the reference (one train-mode pass
with momentum=None), because an uncalibrated random cascade is degenerate (constant depth);
``apply_bn_stats`` installs them.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch


def _key_rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(key.encode())]))


def synthetic_state_dict(template: dict, seed: int = 0) -> dict:
    """Deterministic tensors for every entry of ``template`` (a state_dict or {key: shape})."""
    out = {}
    for k, v in template.items():
        shape = tuple(v.shape) if hasattr(v, "shape") else tuple(v)
        leaf = k.rsplit(".", 1)[-1]
        if leaf == "num_batches_tracked":
            out[k] = torch.zeros((), dtype=torch.long)
            continue
        if leaf == "weight" and len(shape) >= 3:
            fan_in = int(np.prod(shape[1:]))
            arr = _key_rng(seed, k).standard_normal(shape) * np.sqrt(2.0 / fan_in)
        elif leaf in ("weight", "running_var"):
            arr = np.ones(shape)
        else:  # bias, running_mean
            arr = np.zeros(shape)
        out[k] = torch.from_numpy(np.asarray(arr, dtype=np.float32))
    return out


def bn_stat_keys(sd: dict):
    return [k for k in sd if k.endswith(".running_mean") or k.endswith(".running_var")]


def apply_bn_stats(sd: dict, stats: dict) -> dict:
    """Return a copy of ``sd`` with running_mean/var replaced from ``stats`` (numpy or torch)."""
    out = dict(sd)
    for k, v in stats.items():
        if k in out:
            out[k] = torch.as_tensor(np.asarray(v), dtype=torch.float32).reshape(out[k].shape)
    return out
