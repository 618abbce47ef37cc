"""torchaudio.transforms classes (2.7.1 semantics) the reference instantiates."""
import math

import torch

from . import functional as F


class Spectrogram(torch.nn.Module):
    def __init__(self, n_fft=400, win_length=None, hop_length=None, pad=0,
                 window_fn=torch.hann_window, power=2.0, normalized=False, center=True,
                 pad_mode="reflect", onesided=True):
        super().__init__()
        self.n_fft = n_fft
        self.win_length = win_length if win_length is not None else n_fft
        self.hop_length = hop_length if hop_length is not None else self.win_length // 2
        self.register_buffer("window", window_fn(self.win_length))
        self.pad, self.power, self.normalized = pad, power, normalized
        self.center, self.pad_mode, self.onesided = center, pad_mode, onesided

    def forward(self, waveform):
        return F.spectrogram(waveform, self.pad, self.window, self.n_fft, self.hop_length,
                             self.win_length, self.power, self.normalized, self.center,
                             self.pad_mode, self.onesided)


class MelScale(torch.nn.Module):
    def __init__(self, n_mels=128, sample_rate=16000, f_min=0.0, f_max=None, n_stft=201,
                 norm=None, mel_scale="htk"):
        super().__init__()
        f_max = f_max or float(sample_rate // 2)
        self.register_buffer("fb", F.melscale_fbanks(n_stft, f_min, f_max, n_mels, sample_rate,
                                                     norm, mel_scale))

    def forward(self, specgram):
        return torch.matmul(specgram.transpose(-1, -2), self.fb).transpose(-1, -2)


class MelSpectrogram(torch.nn.Module):
    def __init__(self, sample_rate=16000, n_fft=400, win_length=None, hop_length=None,
                 f_min=0.0, f_max=None, pad=0, n_mels=128, window_fn=torch.hann_window,
                 power=2.0, normalized=False, center=True, pad_mode="reflect",
                 onesided=True, norm=None, mel_scale="htk"):
        super().__init__()
        self.spectrogram = Spectrogram(n_fft=n_fft, win_length=win_length,
                                       hop_length=hop_length, pad=pad, window_fn=window_fn,
                                       power=power, normalized=normalized, center=center,
                                       pad_mode=pad_mode, onesided=onesided)
        self.mel_scale = MelScale(n_mels, sample_rate, f_min, f_max, n_fft // 2 + 1, norm,
                                  mel_scale)

    def forward(self, waveform):
        return self.mel_scale(self.spectrogram(waveform))


class AmplitudeToDB(torch.nn.Module):
    def __init__(self, stype="power", top_db=None):
        super().__init__()
        self.stype = stype
        self.top_db = top_db
        self.multiplier = 10.0 if stype == "power" else 20.0
        self.amin = 1e-10
        self.ref_value = 1.0
        self.db_multiplier = math.log10(max(self.amin, self.ref_value))

    def forward(self, x):
        return F.amplitude_to_DB(x, self.multiplier, self.amin, self.db_multiplier, self.top_db)


class _AxisMasking(torch.nn.Module):
    # torchaudio stores the parameter as ``mask_param`` (not time_/freq_mask_param)
    def __init__(self, mask_param, axis, iid_masks=False, p=1.0):
        super().__init__()
        self.mask_param, self.axis, self.iid_masks, self.p = mask_param, axis, iid_masks, p


class TimeMasking(_AxisMasking):
    def __init__(self, time_mask_param, iid_masks=False, p=1.0):
        super().__init__(time_mask_param, 2, iid_masks, p)


class FrequencyMasking(_AxisMasking):
    def __init__(self, freq_mask_param, iid_masks=False):
        super().__init__(freq_mask_param, 1, iid_masks)


class Resample(torch.nn.Module):
    def __init__(self, orig_freq=16000, new_freq=16000, *a, **k):
        super().__init__()
        assert orig_freq == new_freq, "resampling is not restated offline"

    def forward(self, w):
        return w
