"""Reproducibility probe of GpuLogMel (B = 8 ESC-50 clips, the AST test setting): the same call K times, with
and without the per-clip normalisation; reports how many outputs differ from the first and where.
    python tools/logmel_repro.py [K]"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "dl-sound-classification_amd"))
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

from oracle.synth import synth_waveform  # noqa: E402
from src.datasets.features import GpuLogMel  # noqa: E402
from src.miaudio import kernels as K  # noqa: E402
from src.miaudio import lib as L  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
w0 = torch.from_numpy(synth_waveform(71, 8, 220_500)).to(dev)
E = 1 << 20  # guard regions either side of the clips, refilled with garbage every repetition
buf = torch.zeros(w0.numel() + 2 * E, device=dev)
wav = buf[E:E + w0.numel()].view_as(w0)
wav.copy_(w0)
for norm in (False, True):
    lm = GpuLogMel(44_100, 128, norm, 0.0, 0.5)
    ref = lm(wav).clone()
    lib = L.load()
    frames = ref.shape[2]
    bad = 0
    for r in range(reps):
        # garbage in the workspace and the output buffer first: the result must not depend on it
        ws = K.workspace(lib.mia_logmel_workspace_bytes(8, frames), dev, "logmel")
        if r % 3 == 1:
            ws.view(torch.uint8).random_()
        elif r % 3 == 2:
            ws.view(torch.uint8).fill_(0x7f)
        buf[:E].uniform_(-1e3, 1e3)
        buf[E + w0.numel():].uniform_(-1e3, 1e3)
        o = torch.empty_like(ref)
        o.view(torch.int32).random_() if r % 2 else o.fill_(float("nan"))
        o = lm(wav, out=o)
        if not torch.equal(o, ref):
            bad += 1
            d = (o != ref)
            idx = d.nonzero()
            if bad <= 3:
                print(f"normalize={norm} rep {r}: {int(d.sum())} values differ, clips {sorted(set(idx[:, 0].tolist()))}, "
                      f"mels {idx[:, 1].min().item()}..{idx[:, 1].max().item()}, frames {idx[:, 2].min().item()}.."
                      f"{idx[:, 2].max().item()}, max |diff| {float((o - ref).abs().max()):.3g}", flush=True)
    print(f"logmel_repro normalize={norm}: {bad} of {reps} differ", flush=True)
