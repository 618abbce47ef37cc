#!/usr/bin/env python
"""Training entry point — drop-in for the reference scripts/train.py (same config tree, same
override grammar, same flow: seed -> DataModule from dataset config + the model's
``dataset_overrides`` -> LitClassifier via build_from_cfg -> Trainer.fit -> Trainer.test("best");
reference scripts/train.py:55-205).

    python scripts/train.py dataset=esc50 dataset.fold=0 model=envnet_v2
    python scripts/train.py model=ast trainer.precision=bf16-mixed
    python scripts/train.py dataset=synthetic model=envnet_v2 trainer.max_epochs=1
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/train.py trainer.devices=8

Hydra/Lightning/MLflow are not installed in this image: configs are composed by
``src.utils.config.compose`` and metrics go to a JSON-lines logger under ``outputs/``.
"""
from __future__ import annotations

import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.training.engine import build_from_cfg  # noqa: E402
from src.training.lite import CSVLogger, EarlyStopping, ModelCheckpoint, Trainer  # noqa: E402
from src.utils.config import Cfg, compose, instantiate, to_container  # noqa: E402

_DM_KEYS = ("root", "fold", "val_split")
LAST_TRAINER = None  # the Trainer of the latest train() call (tests read its device / process group)


def fix_seed(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def datamodule_config(cfg) -> dict:
    """Same merge as reference train.py:80-115, plus pass-through of extra dataset keys
    (e.g. the synthetic module's num_clips)."""
    ds = cfg.dataset
    dm = {"_target_": ds["_target_"], **{k: ds[k] for k in _DM_KEYS if k in ds},
          "batch_size": cfg.batch_size, "num_workers": cfg.num_workers,
          "num_classes": ds.get("num_classes", 50),
          "enable_bc_mixing": ds.get("enable_bc_mixing", False),
          "enable_mixup": ds.get("enable_mixup", False),
          "mixup_alpha": ds.get("mixup_alpha", 0.5)}
    for k in ("sample_rate", "num_clips", "clip_samples", "seed"):
        if k in ds:
            dm[k] = ds[k]
    overrides = cfg.model.get("dataset_overrides")
    if overrides:
        dm.update(to_container(overrides))
    else:
        dm.update({"preprocessing_mode": ds.get("preprocessing_mode", "envnet_v2"),
                   "preprocessing_config": to_container(ds.get("preprocessing_config", {})),
                   "augment": to_container(ds.get("augment", {})),
                   "is_spectrogram": ds.get("is_spectrogram", False)})
    return dm


def build_callbacks(cfg):
    cbs = []
    if "checkpoint" in cfg:
        cbs.append(ModelCheckpoint(**to_container(cfg.checkpoint)))
    if "early_stop" in cfg:
        cbs.append(EarlyStopping(**to_container(cfg.early_stop)))
    return cbs


def train(cfg) -> dict:
    fix_seed(int(cfg.seed))
    datamodule = instantiate(datamodule_config(cfg))
    model_cfg = {k: v for k, v in cfg.model.items() if k != "dataset_overrides"}
    lit = build_from_cfg(Cfg.wrap({**cfg, "model": model_cfg}))
    logger = CSVLogger(save_dir=os.path.join(ROOT, "outputs"),
                       experiment_name=cfg.get("logging", {}).get("experiment_name", "default"))
    trainer = Trainer(**to_container(cfg.trainer), logger=logger, callbacks=build_callbacks(cfg))
    global LAST_TRAINER
    LAST_TRAINER = trainer
    trainer.fit(lit, datamodule=datamodule, ckpt_path=cfg.get("ckpt_path"))
    out = trainer.test(ckpt_path="best", datamodule=datamodule)
    if trainer.is_global_zero:
        print("training run finished — metrics in", logger.log_dir)
    return out[0]


def launch_ranks(n: int, argv: list[str]) -> int:
    """``trainer.devices=N`` without a launcher: start one process per device through
    torch.distributed.run on this node (rendezvous on 127.0.0.1), as Lightning's DDP strategy re-launches
    the script per rank (reference train.py:190-194).  Runs before this process touches the GPU.  The c10d
    rendezvous store binds port 0 itself (no probe-then-close race for a free port)."""
    import subprocess
    import uuid
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0", f"--rdzv-id={uuid.uuid4()}",
           "--local-addr", "127.0.0.1", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def main(argv=None):
    """Train / test from the config tree.  With ``trainer.devices > 1`` outside a launcher: the launcher's exit
    code (0 = every rank finished); otherwise train()'s result."""
    argv = list(sys.argv[1:] if argv is None else argv)
    cfg = compose(os.path.join(ROOT, "configs"), "training", argv)
    devices = cfg.trainer.get("devices", 1)
    if isinstance(devices, int) and devices > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(devices, argv)
    return train(cfg)


if __name__ == "__main__":
    res = main()
    sys.exit(res if isinstance(res, int) else 0)
