"""CPU tests of the host logic around the hot path: config composition (reference configs tree and
override grammar), DataModule constraint validation (reference esc50.py:437-476), metrics, the
Lightning-compatible loop end to end on a toy model, and the RCCL gradient exchange restated over
gloo with world_size 2."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pathlib import Path
from src.utils.config import compose, instantiate
from src.datasets.esc50 import ESC50DataModule, SyntheticDataModule
from src.training import metrics as M

PKG = Path(__file__).resolve().parents[1] / "dl-sound-classification_amd"
CFG = PKG / "configs"


def test_compose_defaults_and_overrides():
    cfg = compose(CFG, "training", [])
    assert cfg.model["_target_"] == "src.models.ast.ASTModel"
    assert cfg.metric.num_classes == 50  # ${dataset.num_classes} interpolation
    assert cfg.scheduler.T_max == cfg.trainer.max_epochs
    cfg = compose(CFG, "training", ["model=envnet_v2", "dataset.fold=3", "trainer.max_epochs=7", "+ckpt_path=x.ckpt"])
    assert cfg.model["_target_"] == "src.models.envnet_v2.EnvNetV2"
    assert cfg.dataset.fold == 3 and cfg.scheduler.T_max == 7 and cfg.ckpt_path == "x.ckpt"
    assert cfg.model.dataset_overrides.enable_bc_mixing is True
    with pytest.raises(KeyError):
        compose(CFG, "training", ["trainer.not_a_key=1"])


def test_instantiate_scheduler():
    p = torch.nn.Parameter(torch.zeros(2))
    opt = instantiate({"_target_": "torch.optim.Adam", "lr": 0.1}, params=[p])
    sch = instantiate({"_target_": "torch.optim.lr_scheduler.CosineAnnealingLR", "T_max": 4}, optimizer=opt)
    assert isinstance(sch, torch.optim.lr_scheduler.CosineAnnealingLR)


@pytest.mark.parametrize("kw,msg", [
    (dict(is_spectrogram=True, enable_bc_mixing=True), "enable_bc_mixing cannot be true"),
    (dict(is_spectrogram=False, enable_mixup=True), "enable_mixup can only be true"),
    (dict(is_spectrogram=False, time_mask=10), "time_mask will be ignored"),
    (dict(is_spectrogram=True, freq_mask=-3), "freq_mask must be a positive integer"),
])
def test_datamodule_validation(kw, msg):
    with pytest.raises(ValueError, match=msg):
        ESC50DataModule(root="x", **kw)
    with pytest.raises(ValueError):
        ESC50DataModule(root="x", fold=5)


def test_metrics_macro():
    logits = torch.eye(3)[[0, 1, 2, 0, 0]] * 5
    target = torch.tensor([0, 1, 1, 0, 2])
    acc = M.Accuracy(3)
    acc.update(logits, target)
    # per-class recall: c0 2/2, c1 1/2, c2 0/1 -> macro 0.5
    assert abs(float(acc.compute()) - 0.5) < 1e-6
    au = M.AUROC(3)
    au.update(torch.tensor([[3., 0, 0], [0, 3, 0], [0, 0, 3]]), torch.tensor([0, 1, 2]))
    assert abs(float(au.compute()) - 1.0) < 1e-6


def test_esc50_datamodule_files(tmp_path):
    # prepare_esc50.py layout: fold_k/*.pt bundles {"waveform": (1, T), "label": int}
    for f in range(5):
        d = tmp_path / f"fold_{f}"
        d.mkdir()
        for i in range(10):
            torch.save({"waveform": torch.randn(1, 4410), "label": i % 4}, d / f"{i}.pt")
    dm = ESC50DataModule(root=str(tmp_path), fold=2, batch_size=4, num_workers=0, num_classes=4,
                         preprocessing_config={"window_length": 0.1})
    dm.setup("fit")
    assert len(dm._train_set) + len(dm._val_set) == 40 and len(dm._val_set) == 4
    assert len(dm._test_set) == 10
    x, y = next(iter(dm.train_dataloader()))
    assert x.shape == (4, 1, 4410) and y.dtype == torch.int64
    xv, yv = dm.gpu_transform(x, y, training=False)  # no BC mixing on CPU: one-hot labels
    assert yv.shape == (4, 4) and torch.equal(yv.argmax(1), y)


def test_urbansound8k_datamodule_files(tmp_path):
    """UrbanSound8K: ten folds, 10 classes, clips shorter than the 5 s EnvNet window are zero-padded
    into it (pad T/2 each side, crop); fold 10 is out of range; config composes to the class."""
    from src.datasets.urbansound8k import UrbanSound8KDataModule
    with pytest.raises(ValueError, match="ten folds"):
        UrbanSound8KDataModule(root="x", fold=10)
    for f in range(10):
        d = tmp_path / f"fold_{f}"
        d.mkdir()
        for i in range(12):
            torch.save({"waveform": torch.randn(1, 3000), "label": (f + i) % 10}, d / f"{i}.pt")
    dm = UrbanSound8KDataModule(root=str(tmp_path), fold=9, batch_size=5, num_workers=0,
                                preprocessing_config={"window_length": 0.1})  # 4410-sample window > 3000
    dm.setup("fit")
    assert dm.num_classes == 10
    assert len(dm._train_set) + len(dm._val_set) == 108 and len(dm._test_set) == 12
    x, y = next(iter(dm.test_dataloader()))
    assert x.shape == (5, 1, 4410)
    _, yv = dm.gpu_transform(x, y, training=False)
    assert yv.shape == (5, 10)
    cfg = compose(CFG, "training", ["dataset=urbansound8k"])
    assert cfg.dataset["_target_"] == "src.datasets.urbansound8k.UrbanSound8KDataModule"


def test_train_script_toy(tmp_path, monkeypatch):
    import importlib.util
    spec = importlib.util.spec_from_file_location("train_script", PKG / "scripts" / "train.py")
    ts = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ts)
    monkeypatch.chdir(tmp_path)
    cfg = compose(CFG, "training", [
        "dataset=synthetic", "dataset.num_clips=40", "+dataset.clip_samples=64", "dataset.num_classes=5",
        "model=envnet_v2", "trainer.max_epochs=2", "trainer.accelerator=cpu", "batch_size=8", "num_workers=0",
        f"checkpoint.dirpath={tmp_path}/ck"])
    cfg.model = {"_target_": "tests._toy.TinyNet", "num_classes": 5, "in_samples": 64}
    cfg.optimizer.lr = 1e-2
    out = ts.train(cfg)
    assert set(out) >= {"test/acc", "test/f1", "test/auroc", "test/loss"}
    assert list((tmp_path / "ck").glob("*.ckpt"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests._toy import TinyNet
    from src.training.ddp import GradAllReducer
    torch.manual_seed(100 + rank)  # different init per rank: the reducer must broadcast rank 0's
    model = TinyNet(5, 16)
    red = GradAllReducer(model, world, bucket_bytes=256)
    x = torch.randn(8, 16, generator=torch.Generator().manual_seed(7 + rank))
    model(x).square().mean().backward()
    # exercise the early-emission path for one parameter, the rest go through finish()
    first = next(model.parameters())
    model._grad_ready([(first, first.grad.clone())])
    red.finish()
    # numpy payloads: torch tensors would travel as shared-memory handles that vanish when the
    # worker exits before the parent has read them
    q.put((rank, {n: p.detach().numpy().copy() for n, p in model.named_parameters()},
           {n: p.grad.numpy().copy() for n, p in model.named_parameters() if p.grad is not None}, x.numpy().copy()))
    dist.destroy_process_group()


def test_grad_allreducer_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, params, grads, x = q.get(timeout=60)
        res[r] = ({n: torch.from_numpy(v) for n, v in params.items()},
                  {n: torch.from_numpy(v) for n, v in grads.items()}, torch.from_numpy(x))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    p0, g0, _ = res[0]
    p1, g1, _ = res[1]
    for n in p0:
        assert torch.equal(p0[n], p1[n]), n  # rank-0 broadcast
    assert set(g0) == set(g1) and len(g0) == 4
    for n in g0:
        assert torch.allclose(g0[n], g1[n], atol=1e-7), n
    # averaged gradient == gradient of the mean of both ranks' losses on the same weights
    from tests._toy import TinyNet
    m = TinyNet(5, 16)
    m.load_state_dict({**m.state_dict(), **p0}, strict=False)
    loss = sum(m(res[r][2]).square().mean() for r in range(world)) / world
    loss.backward()
    for n, p in m.named_parameters():
        if n not in g0:
            continue
        assert torch.allclose(p.grad, g0[n], atol=1e-6, rtol=1e-5), n
