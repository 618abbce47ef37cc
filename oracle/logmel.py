"""CPU restatement of the reference's AST log-mel transform (TEST INFRASTRUCTURE).

Restates ``ASTPreprocessor.preprocess`` (src/datasets/preprocessing.py:1013-1039,
constants :56-58) together with the third-party pieces it calls, torchaudio 2.7.1
``MelSpectrogram`` + ``AmplitudeToDB`` (uv.lock:2195; torchaudio is absent here,
so its published algorithm is restated):

  stft(n_fft=1024, hop=160, win=hann(400, periodic) zero-padded to 1024 and centred,
       center=True, pad_mode=reflect, onesided) -> |X|^2 (513 bins)
  -> matmul with the htk triangular mel filterbank (f 0..sr//2, 128 mels, norm=None)
  -> 10*log10(clamp(x, 1e-10)) -> max(x, amax_per_clip - 80)     (AmplitudeToDB top_db)
  -> (x - mean) / std_unbiased * target_std + target_mean         (preprocessing.py:1030-1037)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import math

import numpy as np
import torch

N_FFT = 1024
HOP = 160
WIN = 400
N_MELS = 128
SR = 44_100
TOP_DB = 80.0
AMIN = 1e-10


def _hz_to_mel_htk(f):
    return 2595.0 * math.log10(1.0 + f / 700.0)


def mel_fbank(n_freqs: int = N_FFT // 2 + 1, f_min: float = 0.0, f_max: float | None = None,
              n_mels: int = N_MELS, sample_rate: int = SR) -> torch.Tensor:
    """(n_freqs, n_mels) htk filterbank, norm=None (torchaudio.functional.melscale_fbanks)."""
    if f_max is None:
        f_max = float(sample_rate // 2)
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = _hz_to_mel_htk(f_min)
    m_max = _hz_to_mel_htk(f_max)
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down, up))


def hann_periodic(n: int = WIN) -> torch.Tensor:
    return torch.hann_window(n, periodic=True)


def power_spectrogram(wav: torch.Tensor) -> torch.Tensor:
    """(B, T) -> (B, 513, frames) power spectrum."""
    spec = torch.stft(wav, N_FFT, hop_length=HOP, win_length=WIN, window=hann_periodic(WIN),
                      center=True, pad_mode="reflect", normalized=False, onesided=True,
                      return_complex=True)
    return spec.abs().pow(2.0)


def logmel(wav, normalize: bool = True, target_mean: float = 0.0, target_std: float = 0.5,
           n_mels: int = N_MELS, sample_rate: int = SR) -> torch.Tensor:
    """(B, T) float32 waveform -> (B, n_mels, 1 + T//160) normalised log-mel."""
    wav = torch.as_tensor(np.asarray(wav, dtype=np.float32))
    if wav.dim() == 1:
        wav = wav.unsqueeze(0)
    spec = power_spectrogram(wav)
    fb = mel_fbank(n_mels=n_mels, sample_rate=sample_rate)
    mel = torch.matmul(spec.transpose(-1, -2), fb).transpose(-1, -2)
    db = 10.0 * torch.log10(torch.clamp(mel, min=AMIN))
    amax = db.amax(dim=(-2, -1), keepdim=True)
    db = torch.max(db, amax - TOP_DB)
    if normalize:
        out = []
        for b in range(db.shape[0]):
            x = db[b]
            m = x.mean()
            s = x.std()
            if s > 0:
                x = (x - m) / s
                x = x * target_std + target_mean
            out.append(x)
        db = torch.stack(out)
    return db
