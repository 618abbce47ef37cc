"""ESC-50 Dataset / DataModule — drop-in for the reference ``src.datasets.esc50``
(ESC50DataModule ctor kwargs, config-constraint validation, 5-fold split with a stratified
validation split, reference src/datasets/esc50.py:335-629) with the per-clip feature work moved
onto the GPU:

* The Dataset only reads the ``{"waveform": (1, T) f32, "label": int}`` bundles written by
  scripts/prepare_esc50.py (torch.load(weights_only=True)) and, for EnvNet without BC mixing, pads
  T/2 each side and crops (random for training, centre otherwise — preprocessing.py:814-855).
* ``gpu_transform`` runs inside the training step on the device: BC mixing against the resident
  training-set pool (EnvNet) or the batched HIP log-mel -> SpecAugment -> Mixup against the
  resident un-augmented spectrogram pool (AST).  Labels become the same soft (B, C) f32 targets the
  reference produces, so LitClassifier's soft-label loss branch runs as in the reference.
``SyntheticDataModule`` serves device-resident synthetic clips (benchmarks, plumbing runs).
"""
from __future__ import annotations

import math
import random
from pathlib import Path
from typing import Dict, List, Sequence, Union

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset
from torch.utils.data.distributed import DistributedSampler

SR = 44_100


def _one_hot(y: torch.Tensor, C: int) -> torch.Tensor:
    out = torch.zeros(y.numel(), C, dtype=torch.float32, device=y.device)
    out.scatter_(1, y.long().view(-1, 1), 1.0)
    return out


class ESC50Dataset(Dataset):
    def __init__(self, root, folds: Sequence[int] = (), files: List[Path] | None = None, mode: str = "envnet_v2",
                 pad_crop: bool = False, window_length: float = 5.0, padding_ratio: float = 0.5,
                 training: bool = True, multi_crop_test: bool = False, test_crops: int = 10):
        self.root = Path(root)
        if files is not None:
            self.files = list(files)
        else:
            self.files = []
            for f in folds:
                self.files += sorted((self.root / f"fold_{f}").glob("*.pt"))
        if not self.files:
            raise FileNotFoundError(f"No .pt files found in {self.root}; did you run scripts/prepare_esc50.py?")
        self.mode, self.pad_crop, self.training = mode, pad_crop, training
        self.window = int(window_length * SR)
        self.pad = int(self.window * padding_ratio)
        self.multi_crop_test, self.test_crops = multi_crop_test, test_crops

    def __len__(self):
        return len(self.files)

    def load(self, idx):
        b = torch.load(self.files[idx], map_location="cpu", weights_only=True)
        return b["waveform"].float().reshape(1, -1), int(b["label"])

    def _crop(self, w, start):
        return w[..., start:start + self.window]

    def fit_window(self, w):
        """A raw clip as the BC-mixing partner pool holds it: its first ``window`` samples, zero-padded
        on the right when shorter (the reference mixes against the raw partner and truncates both to
        the shorter length, BCMixingUtils.mix_waveforms preprocessing.py:462-466; ESC-50 clips are
        exactly one window, so this is the identity there)."""
        w = w[..., :self.window]
        return torch.nn.functional.pad(w, (0, self.window - w.shape[-1])) if w.shape[-1] < self.window else w

    def __getitem__(self, idx):
        w, label = self.load(idx)
        if self.mode == "envnet_v2" and not self.pad_crop:
            # BC-mixing path: no T/2 padding, but the reference's random_crop still runs
            # (esc50.py:233-234, preprocessing.py:841-855): a shorter clip (UrbanSound8K's <= 4 s) is
            # right-padded to the window, a longer one cropped (random when training, else centred)
            total = w.shape[-1]
            if total <= self.window:
                return torch.nn.functional.pad(w, (0, self.window - total)), label
            start = random.randint(0, total - self.window) if self.training else (total - self.window) // 2
            return self._crop(w, start), label
        if self.mode == "envnet_v2" and self.pad_crop:
            w = torch.nn.functional.pad(w, (self.pad, self.pad))
            total = w.shape[-1]
            if total <= self.window:
                return torch.nn.functional.pad(w, (0, self.window - total)), label
            if not self.training and self.multi_crop_test:
                starts = torch.linspace(0, total - self.window, self.test_crops).long()
                return [self._crop(w, int(s)) for s in starts], label
            start = random.randint(0, total - self.window) if self.training else (total - self.window) // 2
            w = self._crop(w, start)
        return w, label


class ESC50DataModule:
    NUM_FOLDS = 5

    def __init__(self, root: str, fold: int = 0, sample_rate: int = SR, n_mels: int = 128, val_split: float = 0.1,
                 batch_size: int = 32, num_workers: int = 4, is_spectrogram: bool = False,
                 enable_bc_mixing: bool = False, enable_mixup: bool = False, mixup_alpha: float = 0.5,
                 time_mask: Union[bool, int] = False, freq_mask: Union[bool, int] = False,
                 preprocessing_mode: str = "envnet_v2", preprocessing_config: Dict | None = None,
                 num_classes: int = 50, augment: Dict | None = None, **unused):
        if not (0 <= fold < self.NUM_FOLDS):
            raise ValueError(self._fold_error())
        self._validate_config_constraints(is_spectrogram, enable_bc_mixing, enable_mixup, time_mask, freq_mask)
        augment = dict(augment or {})
        if time_mask is not False:
            augment["time_mask"] = time_mask
        if freq_mask is not False:
            augment["freq_mask"] = freq_mask
        self.root, self.fold, self.sample_rate, self.n_mels = root, fold, sample_rate, n_mels
        self.val_split, self.batch_size, self.num_workers = val_split, batch_size, num_workers
        self.is_spectrogram = is_spectrogram
        self.enable_bc_mixing, self.enable_mixup, self.mixup_alpha = enable_bc_mixing, enable_mixup, mixup_alpha
        self.augment = augment
        self.preprocessing_mode = "ast" if is_spectrogram else "envnet_v2"
        self.preprocessing_config = dict(preprocessing_config or {})
        self.num_classes = num_classes
        self.device, self.world, self.rank = torch.device("cpu"), 1, 0
        self._train_set = self._val_set = self._test_set = None
        self._pool = self._pool_labels = None
        self._logmel = None
        self._gen = None

    @classmethod
    def _fold_error(cls) -> str:
        return "fold must be 0…4 (ESC-50 uses five folds)."

    @staticmethod
    def _validate_config_constraints(is_spectrogram, enable_bc_mixing, enable_mixup, time_mask, freq_mask):
        """Same constraints and messages as the reference (esc50.py:437-476)."""
        errors = []
        if is_spectrogram and enable_bc_mixing:
            errors.append("enable_bc_mixing cannot be true when is_spectrogram=true (BC mixing is only for waveform mode)")
        if not is_spectrogram and enable_mixup:
            errors.append("enable_mixup can only be true when is_spectrogram=true (Mixup is only for spectrogram mode)")
        if not is_spectrogram:
            if time_mask is not False and time_mask != 0:
                errors.append("time_mask will be ignored when is_spectrogram=false (SpecAugment is only for spectrogram mode)")
            if freq_mask is not False and freq_mask != 0:
                errors.append("freq_mask will be ignored when is_spectrogram=false (SpecAugment is only for spectrogram mode)")
        if is_spectrogram:
            for name, v in (("time_mask", time_mask), ("freq_mask", freq_mask)):
                if v is not False and not isinstance(v, int):
                    errors.append(f"{name} must be False or a positive integer")
                if isinstance(v, int) and not isinstance(v, bool) and v < 0:
                    errors.append(f"{name} must be a positive integer")
        if errors:
            raise ValueError("Configuration validation failed:\n" + "\n".join(f"  • {e}" for e in errors))

    # -------------------------------------------------------------------- setup
    def attach(self, device, world: int = 1, rank: int = 0):
        self.device, self.world, self.rank = torch.device(device), world, rank

    def _ds(self, **kw):
        pc = self.preprocessing_config
        return ESC50Dataset(self.root, mode=self.preprocessing_mode,
                            window_length=pc.get("window_length", 5.0), padding_ratio=pc.get("padding_ratio", 0.5),
                            multi_crop_test=pc.get("multi_crop_test", False), test_crops=pc.get("test_crops", 10), **kw)

    def setup(self, stage: str | None = None) -> None:
        if self._train_set is not None:
            return
        from sklearn.model_selection import StratifiedShuffleSplit
        train_folds = [f for f in range(self.NUM_FOLDS) if f != self.fold]
        full = self._ds(folds=train_folds, training=True)
        labels = [full.load(i)[1] for i in range(len(full))]
        val_size = math.ceil(len(full) * self.val_split)
        splitter = StratifiedShuffleSplit(n_splits=1, test_size=val_size, random_state=42)
        tr, va = next(splitter.split(np.zeros(len(labels)), labels))
        tr_files = [full.files[i] for i in tr]
        va_files = [full.files[i] for i in va]
        if set(tr_files) & set(va_files):
            raise RuntimeError("Data leakage detected between train and val splits")
        pad_crop = not self.enable_bc_mixing  # reference: BC mixing path skips pad + crop
        self._train_set = self._ds(files=tr_files, training=True, pad_crop=pad_crop)
        self._val_set = self._ds(files=va_files, training=False, pad_crop=True)
        self._test_set = self._ds(folds=[self.fold], training=False, pad_crop=True)
        self._train_labels = [labels[i] for i in tr]

    def _pools(self):
        """Resident augmentation pool on the device (reference preloads it for BC/Mixup, esc50.py:167-187)."""
        if self._pool is not None or not (self.enable_bc_mixing or self.enable_mixup):
            return
        ds = self._train_set
        if self.is_spectrogram:
            waves = torch.stack([ds.load(i)[0][0] for i in range(len(ds))]).to(self.device)
        else:
            waves = torch.stack([ds.fit_window(ds.load(i)[0])[0] for i in range(len(ds))]).to(self.device)
        self._pool_labels = torch.tensor(self._train_labels, dtype=torch.int64, device=self.device)
        if self.is_spectrogram:
            lm = self.logmel()
            self._pool = torch.cat([lm(waves[i:i + 64]) for i in range(0, waves.shape[0], 64)])
        else:
            self._pool = waves

    def logmel(self):
        if self._logmel is None:
            from .features import GpuLogMel
            pc = self.preprocessing_config
            self._logmel = GpuLogMel(self.sample_rate, pc.get("n_mels", self.n_mels), pc.get("normalize", True),
                                     pc.get("target_mean", 0.0), pc.get("target_std", 0.5))
        return self._logmel

    def gpu_transform(self, x: torch.Tensor, y: torch.Tensor, training: bool):
        """Per-batch feature transform + augmentation on the device -> (model input, soft labels)."""
        if isinstance(y, torch.Tensor) and y.dtype != torch.float32:
            y = y.to(self.device)
        if self._gen is None and x.is_cuda:
            self._gen = torch.Generator(device=x.device).manual_seed(1234 + self.rank)
        C = self.num_classes
        if not self.is_spectrogram:
            wav_aug = self.preprocessing_config.get("augment") or {}
            if training and x.is_cuda and (wav_aug.get("time_stretch") or wav_aug.get("gain_shift")):
                # EnvNetPreprocessor.apply_augmentation after the crop, before BC mixing (esc50.py:235-245)
                from .augment import stretch_gain
                x = stretch_gain(x.reshape(x.shape[0], -1), wav_aug.get("time_stretch"), wav_aug.get("gain_shift"),
                                 gen=self._gen).view(x.shape[0], 1, -1)
            if training and self.enable_bc_mixing:
                from .augment import bc_mix, bc_mix_cpu
                self._pools()
                if x.is_cuda:
                    out, ys, _ = bc_mix(x.reshape(x.shape[0], -1), y, C, gen=self._gen, pool=self._pool,
                                        pool_labels=self._pool_labels)
                else:  # trainer.accelerator=cpu (config 1 plumbing) only
                    out, ys, _ = bc_mix_cpu(x, y, C, self._pool, self._pool_labels)
                return out.view(x.shape[0], 1, -1), ys
            return x, _one_hot(y, C)
        spec = self.logmel()(x.reshape(x.shape[0], -1))
        if training:
            from .augment import spec_augment_mixup
            self._pools()
            aug = bool(self.augment.get("time_mask") or self.augment.get("freq_mask"))
            # reference quirk (esc50.py:271-272): the mask sizes read back from torchaudio's
            # TimeMasking/FrequencyMasking fall back to 192 / 48 whatever was configured
            spec, ys = spec_augment_mixup(spec, y, C, 192, 48, self.mixup_alpha, 0.25, gen=self._gen, specaug=aug,
                                          mixup=self.enable_mixup, pool=self._pool, pool_labels=self._pool_labels)
            return spec, ys
        return spec, _one_hot(y, C)

    # -------------------------------------------------------------------- loaders
    def _loader(self, ds, shuffle):
        sampler = DistributedSampler(ds, self.world, self.rank, shuffle=shuffle, seed=42) if self.world > 1 else None
        return DataLoader(ds, batch_size=self.batch_size, shuffle=shuffle and sampler is None, sampler=sampler,
                          num_workers=self.num_workers, pin_memory=self.device.type == "cuda",
                          persistent_workers=self.num_workers > 0)

    def train_dataloader(self):
        if self._train_set is None:
            raise RuntimeError("Dataset not set up. Call setup() first.")
        return self._loader(self._train_set, True)

    def val_dataloader(self):
        if self._val_set is None:
            raise RuntimeError("Dataset not set up. Call setup() first.")
        return self._loader(self._val_set, False)

    def test_dataloader(self):
        if self._test_set is None:
            raise RuntimeError("Dataset not set up. Call setup() first.")
        return self._loader(self._test_set, False)


class _DeviceLoader:
    """Batches straight from device-resident tensors (no host round trip)."""

    def __init__(self, x, y, batch_size, shuffle, seed, world=1, rank=0):
        self.x, self.y, self.bs, self.shuffle, self.seed = x, y, batch_size, shuffle, seed
        self.world, self.rank, self.epoch = world, rank, 0

    def set_epoch(self, e):
        self.epoch = e

    def _index(self):
        n = self.x.shape[0]
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        return idx[self.rank::self.world]

    def __len__(self):
        return max(1, math.ceil(len(self._index()) / self.bs))

    def __iter__(self):
        idx = self._index().to(self.x.device)
        for i in range(0, idx.numel(), self.bs):
            j = idx[i:i + self.bs]
            yield self.x[j], self.y[j]


class SyntheticDataModule(ESC50DataModule):
    """Device-resident synthetic clips with the ESC-50 DataModule interface: 0.1*N(0,1), peak-normalised
    (prepare_esc50.py:98-101), uniform labels; split into train/val/test 80/10/10."""

    def __init__(self, root: str = "none", num_clips: int = 64, clip_samples: int = 220_500, seed: int = 0, **kw):
        kw.pop("fold", None)
        super().__init__(root=root, fold=0, **kw)
        self.num_clips, self.clip_samples, self.seed = num_clips, clip_samples, seed

    def setup(self, stage=None):
        if self._train_set is not None:
            return
        g = torch.Generator(device=self.device).manual_seed(self.seed)
        x = 0.1 * torch.randn(self.num_clips, 1, self.clip_samples, generator=g, device=self.device)
        x = x / x.abs().amax(dim=-1, keepdim=True)
        y = torch.randint(0, self.num_classes, (self.num_clips,), generator=g, device=self.device)
        n = self.num_clips
        nv = max(1, n // 10)
        self._train_set = (x[: n - 2 * nv], y[: n - 2 * nv])
        self._val_set = (x[n - 2 * nv: n - nv], y[n - 2 * nv: n - nv])
        self._test_set = (x[n - nv:], y[n - nv:])
        self._train_labels = self._train_set[1].tolist()

    def _pools(self):
        if self._pool is not None or not (self.enable_bc_mixing or self.enable_mixup):
            return
        waves, labels = self._train_set
        self._pool_labels = labels
        self._pool = self.logmel()(waves.reshape(waves.shape[0], -1)) if self.is_spectrogram \
            else waves.reshape(waves.shape[0], -1)

    def train_dataloader(self):
        return _DeviceLoader(*self._train_set, self.batch_size, True, 42, self.world, self.rank)

    def val_dataloader(self):
        return _DeviceLoader(*self._val_set, self.batch_size, False, 42, self.world, self.rank)

    def test_dataloader(self):
        return _DeviceLoader(*self._test_set, self.batch_size, False, 42, self.world, self.rank)
