"""Deterministic, RNG-free parameter fill shared by the golden-fixture generator
and the parity tests.

No `droid.pth` exists offline, and torch's RNG init order is not stable across
versions, so UpdateModule weights are a pure function of (parameter name,
shape): a scaled sine sequence.  The generator (make_golden.py) applies it to
the reference's own `droid_net.UpdateModule`; the tests apply it to ours.
"""
import math

import numpy as np


def _name_phase(name: str) -> float:
    return (sum((i + 1) * ord(c) for i, c in enumerate(name)) % 997) / 97.0


def fill_array(name: str, shape) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    idx = np.arange(n, dtype=np.float64)
    vals = np.sin(idx * 0.7311 + _name_phase(name))
    if len(shape) >= 2:
        fan_in = n // shape[0]
        scale = 1.0 / math.sqrt(fan_in)
    else:
        scale = 0.05
    return (vals * scale).reshape(shape).astype(np.float32)


def det_fill(module) -> None:
    """Fill every parameter of a torch module in place."""
    import torch
    with torch.no_grad():
        for name, p in module.named_parameters():
            p.copy_(torch.from_numpy(fill_array(name, tuple(p.shape))))


def det_state_dict(shapes: dict) -> dict:
    """name -> float32 array, for a {name: shape} mapping."""
    return {k: fill_array(k, tuple(v)) for k, v in shapes.items()}
