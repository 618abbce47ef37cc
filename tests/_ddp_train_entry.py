"""Per-rank entry for tests/test_gpu_ddp_train_script.py: runs the drop-in scripts/train.py (``main``) under
torch.distributed.run and records what the rank did, as JSON in ``<out>/rank<r>.json``:

* every index list a DistributedSampler yielded (dataset length, shuffle flag, epoch, indices) -- the
  shard this rank actually trained / validated / tested on;
* the returned test metrics;
* the world size and backend of the process group.

usage: python -m torch.distributed.run ... tests/_ddp_train_entry.py <out_dir> <override> ...
"""
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))

from torch.utils.data.distributed import DistributedSampler  # noqa: E402

SEEN = []
_iter = DistributedSampler.__iter__


def _recording_iter(self):
    idx = list(_iter(self))
    SEEN.append({"n": len(self.dataset), "shuffle": bool(self.shuffle), "epoch": int(self.epoch), "idx": idx})
    return iter(idx)


DistributedSampler.__iter__ = _recording_iter


def main():
    out = Path(sys.argv[1])
    import importlib.util
    spec = importlib.util.spec_from_file_location("train_script", REPO / "dl-sound-classification_amd" / "scripts"
                                                  / "train.py")
    ts = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ts)
    metrics = ts.main(sys.argv[2:])
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    rec = {"rank": rank, "world": dist.get_world_size() if dist.is_initialized() else 1,
           "backend": dist.get_backend() if dist.is_initialized() else None,
           "metrics": metrics, "sampled": SEEN, "device": str(ts.LAST_TRAINER.device)}
    out.mkdir(parents=True, exist_ok=True)
    (out / f"rank{rank}.json").write_text(json.dumps(rec))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
