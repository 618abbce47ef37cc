"""UrbanSound8K DataModule (BASELINE configs 4-5).

The reference has no UrbanSound8K loader (only download_data.py:84-87; TRAINING.md:68-69 names a
``dataset=urbansound8k`` config that does not exist), so this follows the ESC-50 DataModule it would
sit beside: the same ``{"waveform": (1, T) f32 peak-normalised, "label": int}`` bundles under
``root/fold_<k>/`` (k = 0..9 for the dataset's ten predefined folds, clips resampled to 44.1 kHz
by the preparation step), the same constructor arguments and config constraints, one held-out test
fold, a stratified validation split of the other nine, and the EnvNet pad + crop to the 5 s window
(US8K clips are at most 4 s, so the crop window always contains the clip plus zero padding).
Labels are the 10 US8K classes; everything on the device (BC mixing, log-mel, SpecAugment, Mixup)
is shared with ESC-50.
"""
from __future__ import annotations

from .esc50 import ESC50DataModule


class UrbanSound8KDataModule(ESC50DataModule):
    NUM_FOLDS = 10

    def __init__(self, root: str, fold: int = 0, num_classes: int = 10, **kw):
        super().__init__(root=root, fold=fold, num_classes=num_classes, **kw)

    @classmethod
    def _fold_error(cls) -> str:
        return "fold must be 0…9 (UrbanSound8K uses ten folds)."
