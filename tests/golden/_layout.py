"""Inputs of the split / multi-crop fixtures shared by make_golden.py (which writes them with the
reference's code) and the tests that replay them (no path manipulation, no reference imports)."""
import numpy as np

from oracle.synth import hash_uniform

SAMPLE_IDX_SEED = 555
SPLIT_FOLD_CLIPS, SPLIT_CLASSES, SPLIT_TEST_FOLD = 24, 6, 2
MCROP_CASES = [(0.5, 22050, 10), (0.5, 15000, 10), (0.25, 20000, 4)]  # (window s, clip samples, test_crops)


def split_label(fold: int, i: int) -> int:
    """Label of clip i of fold `fold` in the split fixture's synthetic ESC-50 layout."""
    return (7 * fold + 5 * i + (i * i) % 3) % SPLIT_CLASSES


def mcrop_clip(s: int) -> np.ndarray:
    return hash_uniform(6000 + s, (1, MCROP_CASES[s][1])).astype(np.float32)


def sample_idx(n, k, seed=SAMPLE_IDX_SEED):
    return (hash_uniform(seed, (k,), 0.0, 1.0) * n).astype(np.int64).clip(0, n - 1)


def checksum(a: np.ndarray, k: int = 64, seed: int = SAMPLE_IDX_SEED):
    a = np.asarray(a, dtype=np.float64).ravel()
    idx = sample_idx(a.size, k, seed)
    return {"sum": a.sum(), "sumsq": (a * a).sum(), "idx": idx, "vals": a[idx]}
