"""Batched on-GPU log-mel (the AST feature transform) — replaces the per-clip CPU
``ASTPreprocessor.preprocess`` (reference src/datasets/preprocessing.py:971-1039) with one
fused kernel launch over a (B, T) waveform batch already resident in HBM.

The constant tables (periodic Hann window, FFT twiddles, sparse htk mel bands) are built once
per device on the host, following torchaudio 2.7.1 ``melscale_fbanks(norm=None, mel_scale='htk')``
(the filterbank the reference instantiates at preprocessing.py:988-995), and copied to HBM.
"""
from __future__ import annotations

import math

import torch

from ..miaudio import kernels as K
from ..miaudio import lib as L

AST_N_FFT = 1024
AST_HOP_LENGTH = 160
AST_WIN_LENGTH = 400


def htk_mel_filterbank(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int) -> torch.Tensor:
    """(n_freqs, n_mels) triangular filterbank, float32, computed like torchaudio 2.7.1."""
    def hz_to_mel(f):
        return 2595.0 * math.log10(1.0 + f / 700.0)
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(hz_to_mel(f_min), hz_to_mel(f_max), n_mels + 2)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down, up))


class GpuLogMel:
    """``out = logmel(wav)``: (B, T) f32 CUDA -> (B, n_mels, 1 + T // 160) f32 CUDA."""

    def __init__(self, sample_rate: int = 44100, n_mels: int = 128, normalize: bool = True,
                 target_mean: float = 0.0, target_std: float = 0.5, top_db: float = 80.0):
        self.cfg = L.MiaMelCfg(sample_rate, AST_N_FFT, AST_WIN_LENGTH, AST_HOP_LENGTH, n_mels, int(normalize),
                               top_db, target_mean, target_std)
        self.n_mels = n_mels
        fb = htk_mel_filterbank(AST_N_FFT // 2 + 1, 0.0, float(sample_rate // 2), n_mels, sample_rate)
        starts, lens, offs, ws = [], [], [], []
        for m in range(n_mels):
            nz = torch.nonzero(fb[:, m] != 0).flatten()
            if nz.numel() == 0:
                starts.append(0), lens.append(0), offs.append(len(ws))
                continue
            k0, k1 = int(nz[0]), int(nz[-1]) + 1
            starts.append(k0), lens.append(k1 - k0), offs.append(len(ws))
            ws.extend(fb[k0:k1, m].tolist())
        self._host = {
            "window": torch.hann_window(AST_WIN_LENGTH, periodic=True, dtype=torch.float32),
            "tw512": torch.view_as_real(torch.exp(-2j * math.pi * torch.arange(512, dtype=torch.float64) / 512)
                                        ).float().contiguous(),
            "tw1024": torch.view_as_real(torch.exp(-2j * math.pi * torch.arange(513, dtype=torch.float64) / 1024)
                                         ).float().contiguous(),
            "band_start": torch.tensor(starts, dtype=torch.int32),
            "band_len": torch.tensor(lens, dtype=torch.int32),
            "band_off": torch.tensor(offs, dtype=torch.int32),
            "band_w": torch.tensor(ws if ws else [0.0], dtype=torch.float32),
        }
        self.nnz = len(ws)
        self._dev = {}

    def tables(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = {k: v.to(device) for k, v in self._host.items()}
        return self._dev[key]

    def __call__(self, wav: torch.Tensor, out: torch.Tensor | None = None, lib=None) -> torch.Tensor:
        """``lib``: another build of the C ABI (tools/bench_logmel.py A/B); default the product library."""
        L.require_device(wav, "GpuLogMel")
        if wav.dim() == 3:
            wav = wav.reshape(wav.shape[0], -1)
        wav = wav.contiguous().float()
        B, T = wav.shape
        frames = 1 + T // AST_HOP_LENGTH
        if out is None:
            out = torch.empty(B, self.n_mels, frames, dtype=torch.float32, device=wav.device)
        t = self.tables(wav.device)
        lib = lib or L.load()
        ws = K.workspace(lib.mia_logmel_workspace_bytes(B, frames), wav.device, "logmel")
        # algorithmic HBM bytes: waveform read once + log-mel written once, f32
        with K.probe("logmel.fwd", 0.0, B * T * 4 + out.numel() * 4):
            L.check(lib.mia_logmel_fwd(wav.data_ptr(), B, T, T, self.cfg, t["window"].data_ptr(),
                                       t["tw512"].data_ptr(), t["tw1024"].data_ptr(), t["band_start"].data_ptr(),
                                       t["band_len"].data_ptr(), t["band_off"].data_ptr(), t["band_w"].data_ptr(),
                                       out.data_ptr(), ws.data_ptr(), K.logmel_err_word(wav.device).data_ptr(),
                                       L.stream_ptr()), "mia_logmel_fwd")
        return out
