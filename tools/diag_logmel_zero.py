"""Diagnose the log-mel path on a quiet clip + an all-zero clip: raw dB (normalize off), block maxima,
normalised output, against the oracle."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "dl-sound-classification_amd")]
import numpy as np, torch
from oracle import logmel as olog
from oracle.synth import synth_waveform
from src.datasets.features import GpuLogMel
from src.miaudio import kernels as K
wav = np.stack([synth_waveform(3, 1, 20_000)[0] * 1e-4, np.zeros(20_000, np.float32)])
wav[0, 5000:15000] = 0.0
d = torch.from_numpy(wav).cuda()
raw = GpuLogMel(normalize=False)(d).cpu().numpy()
ref_raw = olog.logmel(wav, normalize=False).numpy()
print("raw clip1 min/max", raw[1].min(), raw[1].max(), "ref", ref_raw[1].min(), ref_raw[1].max())
print("raw clip0 min/max", raw[0].min(), raw[0].max(), "ref", ref_raw[0].min(), ref_raw[0].max())
print("raw err per clip", np.abs(raw - ref_raw).reshape(2, -1).max(1))
bad = np.argwhere(np.abs(raw[1] - ref_raw[1]) > 1e-3)
print("clip1 bad count", len(bad), bad[:10], "distinct clip1 values", np.unique(raw[1])[:8])
ws = K._WS[(str(d.device), "logmel")]
print("blockmax", ws[:64].view(torch.float32).cpu().numpy())
out = GpuLogMel()(d).cpu().numpy()
ref = olog.logmel(wav).numpy()
print("norm err per clip", np.abs(out - ref).reshape(2, -1).max(1), out[1].min(), out[1].max())
