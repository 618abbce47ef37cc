"""In-process A/B of a module-level switch of the AST path on the bench's AST train step (B=256): the step
is timed alternately with the switch off and on (FLAG=module:attribute, default
src.models.ast_hip:ATTN_SAVE_Q).
    python tools/ab_ast_flag.py"""
import importlib
import os
import sys
import types
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
import torch  # noqa: E402

from bench_ast import build_ast_step  # noqa: E402

modname, attr = os.environ.get("FLAG", "src.models.ast_hip:ATTN_SAVE_Q").split(":")
mod = importlib.import_module(modname)
dev = torch.device("cuda:0")
B = int(os.environ.get("BATCH", 256))
step, _, _, _ = build_ast_step(types.SimpleNamespace(dtype=os.environ.get("DTYPE", "bf16")), dev, 0, 1, B)
for _ in range(2):
    step()
torch.cuda.synchronize()
res = {False: [], True: []}
for _ in range(int(os.environ.get("ROUNDS", 3))):
    for flag in (False, True):
        setattr(mod, attr, flag)
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            step()
        e1.record()
        torch.cuda.synchronize()
        res[flag].append(e0.elapsed_time(e1) / 3)
        print(f"{attr}={flag}: {res[flag][-1]:.2f} ms/step", flush=True)
for flag, ts in res.items():
    print(f"{attr}={flag}: best {min(ts):.2f} ms/step = {B * 1000 / min(ts):.1f} clips/s", flush=True)
