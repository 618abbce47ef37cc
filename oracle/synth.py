"""Counter-based synthetic data for parity fixtures (TEST INFRASTRUCTURE).

ORACLE HEADER: everything under ``oracle/`` is a CPU restatement of the
reference path used ONLY as a checker by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py``.  The product path never imports it.

Values come from splitmix64(counter) so the same tensors are regenerated
bit-identically in this container and on the GPU box, independent of the
torch / numpy RNG streams (SURVEY.md §8c "Fixtures to commit").
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_SEEDMUL = np.uint64(0xD1B54A32D192ED03)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def hash_uniform(seed: int, shape, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """float32 array of ``shape`` with values in [lo, hi), a pure function of (seed, index)."""
    shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
    n = int(np.prod(shape)) if shape else 1
    out = np.empty(n, dtype=np.float32)
    with np.errstate(over="ignore"):
        key = np.uint64(seed) * _SEEDMUL
    chunk = 1 << 24
    scale = np.float32(hi - lo)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        idx = np.arange(s, e, dtype=np.uint64) ^ key
        z = _splitmix64(idx)
        u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))
        out[s:e] = np.float32(lo) + scale * u
    return out.reshape(shape)


def hash_labels(seed: int, n: int, num_classes: int) -> np.ndarray:
    """int64 labels uniform in [0, num_classes)."""
    with np.errstate(over="ignore"):
        key = np.uint64(seed) * _SEEDMUL
    z = _splitmix64(np.arange(n, dtype=np.uint64) ^ key)
    return (z % np.uint64(num_classes)).astype(np.int64)


def synth_waveform(seed: int, batch: int, T: int = 220_500) -> np.ndarray:
    """(batch, T) float32 clips, per-clip peak-normalised to max|x| = 1
    (mirrors scripts/prepare_esc50.py:98-101 peak normalisation)."""
    w = hash_uniform(seed, (batch, T))
    peak = np.abs(w).max(axis=1, keepdims=True)
    peak[peak == 0] = 1.0
    return (w / peak).astype(np.float32)
