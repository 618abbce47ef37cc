"""GPU: config 4's data-parallel leg through the drop-in, rehearsed on one GPU.

``scripts/train.py model=envnet_v2 dataset=urbansound8k trainer.devices=2 trainer.dist_backend=gloo``
launched through torch.distributed.run (reference scripts/train.py:190-201 with
configs/base_training.yaml:45-49: Lightning re-launches the script per rank under DDPStrategy).  The two
ranks share the one GPU (gloo carries the GPU tensors; RCCL refuses two ranks on one device): each joins
the process group, trains its DistributedSampler shard with GradAllReducer exchanging the gradients,
rank 0 writes the one checkpoint, both test the best checkpoint with the metric states synchronised.
Then the same command resumes from that checkpoint for one more epoch.

What is checked, from what each rank recorded (tests/_ddp_train_entry.py):
* the train shards of every epoch are disjoint across ranks and together cover the train set (up to
  DistributedSampler's even-length padding), and reshuffle between epochs;
* exactly one checkpoint file exists (rank 0's), holding replace_head(10)'s head;
* test/acc, test/f1 and test/auroc -- synchronised across ranks, as torchmetrics does at compute() --
  are the same on both ranks (test/loss is per rank, as the reference logs it without sync_dist,
  engine.py:186);
* the resumed run continues at the epoch after the checkpoint's, on both ranks, with finite metrics.
"""
import json
import math
import os
import subprocess
import sys
from pathlib import Path

import pytest

from tests.test_gpu_train_script import _us8k_tree
from tests.test_training_cpu import _free_port

REPO = Path(__file__).resolve().parents[1]


def _run(tmp_path, out, extra, timeout=420, device_args=("trainer.precision=bf16-mixed", "trainer.dist_backend=gloo")):
    env = dict(os.environ, MIA_QUIET="1", PYTHONPATH=str(REPO))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           str(REPO / "tests" / "_ddp_train_entry.py"), str(out),
           "dataset=urbansound8k", f"dataset.root={tmp_path}/us8k", "dataset.fold=9", "model=envnet_v2",
           *device_args, "trainer.devices=2", "batch_size=8", "num_workers=0", f"checkpoint.dirpath={tmp_path}/ck", "checkpoint.monitor=val/loss",
           "checkpoint.mode=min", *extra]
    p = subprocess.run(cmd, cwd=tmp_path, env=env, timeout=timeout, capture_output=True, text=True)
    print(p.stdout[-4000:])
    print(p.stderr[-4000:], file=sys.stderr)
    assert p.returncode == 0, p.stderr[-3000:]
    recs = [json.loads((out / f"rank{r}.json").read_text()) for r in range(2)]
    assert all(r["world"] == 2 and r["backend"] == "gloo" for r in recs)
    assert all(r["device"].startswith("cuda" if "trainer.dist_backend=gloo" in device_args else "cpu") for r in recs)
    return recs


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_train_script_envnet_us8k_two_ranks_gloo(cuda, tmp_path):
    _check(tmp_path, [])


@pytest.mark.timeout(600)
def test_train_script_envnet_us8k_two_ranks_cpu(tmp_path):
    """The same launch on the CPU (trainer.accelerator=cpu: config 1's torch-CPU plumbing, gloo process group),
    one batch per stage, so the N > 1 drop-in path is covered by the CPU suite too."""
    _check(tmp_path, ["batch_size=4", "+trainer.limit_train_batches=1", "+trainer.limit_val_batches=1",
                      "+trainer.limit_test_batches=1"], device_args=("trainer.accelerator=cpu",))


def _check(tmp_path, extra, **kw):
    import torch
    _us8k_tree(tmp_path)
    recs = _run(tmp_path, tmp_path / "run1", ["trainer.max_epochs=2", *extra], **kw)
    train = [[s for s in r["sampled"] if s["shuffle"]] for r in recs]
    assert len(train[0]) == len(train[1]) == 2  # one shuffled train pass per epoch per rank
    n = train[0][0]["n"]
    for e in range(2):
        a, b = train[0][e]["idx"], train[1][e]["idx"]
        assert train[0][e]["epoch"] == train[1][e]["epoch"] == e
        assert len(a) == len(b) == math.ceil(n / 2)
        assert set(a) | set(b) == set(range(n))
        assert len(set(a) & set(b)) <= 2 * math.ceil(n / 2) - n  # only DistributedSampler's padding repeats
    assert train[0][0]["idx"] != train[0][1]["idx"], "the shard order must change with the epoch"
    ck = sorted((tmp_path / "ck").glob("*.ckpt"))
    assert len(ck) == 1, ck
    saved = torch.load(ck[0], map_location="cpu", weights_only=True)
    assert saved["state_dict"]["model.classifier.7.weight"].shape == (10, 4096)
    m0, m1 = recs[0]["metrics"], recs[1]["metrics"]
    for k in ("test/acc", "test/f1", "test/auroc"):
        assert k in m0 and m0[k] == m1[k], (k, m0.get(k), m1.get(k))
    assert all(math.isfinite(v) for r in recs for v in r["metrics"].values())
    start = saved["epoch"] + 1  # fit(ckpt_path) resumes after the checkpoint's epoch, for one more epoch
    recs2 = _run(tmp_path, tmp_path / "run2", [f"trainer.max_epochs={start + 1}", f"+ckpt_path={ck[0]}", *extra],
                 **kw)
    resumed = [[s for s in r["sampled"] if s["shuffle"]] for r in recs2]
    assert [s["epoch"] for s in resumed[0]] == [start] == [s["epoch"] for s in resumed[1]]
    assert all(math.isfinite(v) for r in recs2 for v in r["metrics"].values())
