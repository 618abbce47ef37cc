"""torchaudio.functional pieces (2.7.1 semantics) used by MelSpectrogram/AmplitudeToDB."""
import math

import torch


def _hz_to_mel(f):
    return 2595.0 * math.log10(1.0 + f / 700.0)


def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate, norm=None, mel_scale="htk"):
    assert norm is None and mel_scale == "htk"
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(_hz_to_mel(f_min), _hz_to_mel(f_max), n_mels + 2)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down_slopes = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up_slopes = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down_slopes, up_slopes))


def spectrogram(waveform, pad, window, n_fft, hop_length, win_length, power, normalized,
                center=True, pad_mode="reflect", onesided=True):
    shape = waveform.size()
    waveform = waveform.reshape(-1, shape[-1])
    spec_f = torch.stft(waveform, n_fft=n_fft, hop_length=hop_length, win_length=win_length,
                        window=window, center=center, pad_mode=pad_mode, normalized=False,
                        onesided=onesided, return_complex=True)
    spec_f = spec_f.reshape(shape[:-1] + spec_f.shape[-2:])
    if power is None:
        return spec_f
    if power == 1.0:
        return spec_f.abs()
    return spec_f.abs().pow(power)


def amplitude_to_DB(x, multiplier, amin, db_multiplier, top_db=None):
    x_db = multiplier * torch.log10(torch.clamp(x, min=amin))
    x_db -= multiplier * db_multiplier
    if top_db is not None:
        shape = x_db.size()
        packed_channels = shape[-3] if x_db.dim() > 2 else 1
        x_db = x_db.reshape(-1, packed_channels, shape[-2], shape[-1])
        x_db = torch.max(x_db, (x_db.amax(dim=(-3, -2, -1)) - top_db).view(-1, 1, 1, 1))
        x_db = x_db.reshape(shape)
    return x_db
