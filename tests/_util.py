"""Shared helpers for the parity tests (the oracle is used only as the checker)."""
import numpy as np
import torch

from oracle import envnet as oenv


_PARAMS = {}


def hash_params(seed=100):
    if seed not in _PARAMS:
        _PARAMS[seed] = oenv.hash_params(seed)
    return _PARAMS[seed]


def envnet_with_hash_params(device, dropout=0.0, compute_dtype="f32", seed=100):
    from src.models.envnet_v2 import EnvNetV2
    m = EnvNetV2(num_classes=50, dropout=dropout, compute_dtype=compute_dtype)
    sd = {k: torch.from_numpy(v.copy()) for k, v in hash_params(seed).items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected and all(k.endswith("num_batches_tracked") for k in missing)
    return m.to(device)


def sampled(a, idx):
    return np.asarray(a, dtype=np.float64).ravel()[idx]


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)
