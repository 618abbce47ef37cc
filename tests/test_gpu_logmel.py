"""GPU: fused log-mel kernel vs the oracle (torch.stft restatement of torchaudio 2.7.1 +
ASTPreprocessor normalisation) and the reference's golden outputs.
Tolerance: 2e-4 absolute on the normalised (std 0.5) log-mel — f32 FFT vs pocketfft rounding."""
import numpy as np
import pytest
import torch

from oracle import logmel as olog
from oracle.synth import hash_uniform, synth_waveform
from src.datasets.features import GpuLogMel

pytestmark = pytest.mark.gpu
ATOL = 2e-4


def test_short_clips_vs_golden(cuda, golden):
    wav = torch.from_numpy(synth_waveform(11, 2, 16_000)).to(cuda)
    out = GpuLogMel()(wav).cpu().numpy()
    assert out.shape == (2, 128, 101)
    np.testing.assert_allclose(out, golden["logmel_short"], atol=ATOL, rtol=0)


def test_unnormalised_db_vs_golden(cuda, golden):
    wav = torch.from_numpy(synth_waveform(11, 1, 16_000)).to(cuda)
    out = GpuLogMel(normalize=False)(wav).cpu().numpy()[0]
    np.testing.assert_allclose(out, golden["logmel_short_db"], atol=5e-3, rtol=0)


def test_full_clips_vs_golden_checksums(cuda, golden):
    wav = torch.from_numpy(synth_waveform(12, 2, 220_500)).to(cuda)
    out = GpuLogMel()(wav).cpu().numpy()
    assert out.shape == (2, 128, 1379)
    for b in range(2):
        idx = golden[f"logmel_full{b}__idx"]
        np.testing.assert_allclose(out[b].ravel()[idx], golden[f"logmel_full{b}__vals"], atol=ATOL)
        np.testing.assert_allclose(out[b].mean(axis=1), golden[f"logmel_full{b}__rowmean"], atol=ATOL)


@pytest.mark.parametrize("T", [600, 5000, 44_100, 220_500 + 37])
def test_ragged_lengths_vs_oracle(cuda, T):
    wav = synth_waveform(T, 3, T)
    ref = olog.logmel(wav).numpy()
    out = GpuLogMel()(torch.from_numpy(wav).to(cuda)).cpu().numpy()
    assert out.shape == ref.shape
    np.testing.assert_allclose(out, ref, atol=ATOL, rtol=0)


def test_quiet_and_silent_rows(cuda):
    # a near-silent clip exercises the top_db clamp; an all-zero clip has std 0 (no normalisation)
    wav = np.stack([synth_waveform(3, 1, 20_000)[0] * 1e-4, np.zeros(20_000, np.float32)])
    wav[0, 5000:15000] = 0.0
    ref = olog.logmel(wav).numpy()
    out = GpuLogMel()(torch.from_numpy(wav).to(cuda)).cpu().numpy()
    np.testing.assert_allclose(out, ref, atol=ATOL, rtol=0)


def test_batch256_properties(cuda):
    """Full-size batch: every clip normalised to mean 0 / unbiased std 0.5, row 0 constant."""
    wav = torch.from_numpy(hash_uniform(77, (256, 220_500))).to(cuda)
    out = GpuLogMel()(wav)
    m = out.mean(dim=(1, 2))
    s = out.flatten(1).std(dim=1)
    assert float(m.abs().max()) < 1e-4
    assert float((s - 0.5).abs().max()) < 1e-4
    assert float((out[:, 0, :] - out[:, 0, :1]).abs().max()) == 0.0
    ref = olog.logmel(wav[:2].cpu().numpy()).numpy()
    np.testing.assert_allclose(out[:2].cpu().numpy(), ref, atol=ATOL)
