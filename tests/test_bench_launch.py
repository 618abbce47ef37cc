"""CPU: bench.py's multi-rank plumbing.  ``python bench.py --gpus N`` without a launcher starts N ranks
itself through torch.distributed.run (``bench.launch_ranks``, before anything touches a GPU), and every
rank refuses to time a process group whose size differs from --gpus (``bench.check_world``).  The
script launched here is a stand-in rank with the same rendezvous (127.0.0.1, gloo on CPU); the bench
itself needs the GPU."""
import json
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import bench  # noqa: E402

RANK_SCRIPT = '''
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
assert dist.get_world_size() == int(os.environ["WORLD_SIZE"])
if dist.get_rank() == 0:
    print(json.dumps({"n_gpus": dist.get_world_size(), "sum": float(t), "argv": sys.argv[1:]}), flush=True)
dist.destroy_process_group()
'''


def test_launch_ranks_runs_n_ranks_and_forwards_argv(tmp_path, capfd):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    rc = bench.launch_ranks(2, str(script), ["--gpus", "2", "--steps", "3"])
    assert rc == 0
    lines = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, "rank 0 alone prints the line"
    out = json.loads(lines[0])
    assert out == {"n_gpus": 2, "sum": 3.0, "argv": ["--gpus", "2", "--steps", "3"]}


def test_launch_ranks_propagates_failure(tmp_path):
    script = tmp_path / "bad.py"
    script.write_text("import sys; sys.exit(3)\n")
    assert bench.launch_ranks(2, str(script), []) != 0


def test_check_world():
    bench.check_world(None, 4)
    bench.check_world(2, 2)
    with pytest.raises(SystemExit):
        bench.check_world(8, 1)


def test_attention_summary_credited_and_counter_figures():
    """The AST legs' attention object: credited rate from the probed launches (forward + backward FLOPs of
    SURVEY §8(d) over their live time) and the MFMA-busy figures of the committed SQ profile."""
    ks = {"attn.fwd": {"ms": 2.0, "launches_per_step": 12.0, "flop": 2.0e12},
          "attn.bwd": {"ms": 6.0, "launches_per_step": 12.0, "flop": 4.0e12}}
    res = bench.attention_summary("ast", ks, 2500.0)
    assert res["credited_tflops"] == 750.0 and res["credited_frac"] == 0.3 and res["ms_per_step"] == 96.0
    busy = res["mfma_busy"]
    assert busy["source"].endswith("_sq_ast.json")
    assert set(busy["kernels"]) == set(bench.ATTN_KERNELS)
    assert all(0.0 < k["mfma_busy"] < 1.0 for k in busy["kernels"].values())
    assert 0.0 < busy["time_weighted"] < 1.0
    assert bench.attention_summary("ast", {}, 2500.0)["mfma_busy"]  # counters alone when nothing was probed
