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


# ---- the in-kernel FFT self-check (Parseval + the vanishing lag-512 autocorrelation of the power spectrum) ----
def _fresh_err_word(monkeypatch, cuda):
    from src.miaudio import kernels as K
    w = torch.zeros(8, dtype=torch.int32, device=cuda)
    monkeypatch.setitem(K._LOGMEL_ERR, str(cuda), w)
    return w


def test_self_check_silent_on_clean_batches(cuda, monkeypatch):
    """Full-size clips, ragged and near-silent rows: no frame fails or is retried, and two calls agree bit for bit."""
    w = _fresh_err_word(monkeypatch, cuda)
    wav = torch.from_numpy(hash_uniform(78, (64, 220_500))).to(cuda)
    mel = GpuLogMel()
    a = mel(wav)
    b = mel(wav)
    quiet = np.stack([synth_waveform(3, 1, 20_000)[0] * 1e-4, np.zeros(20_000, np.float32)])
    mel(torch.from_numpy(quiet).to(cuda))
    GpuLogMel(normalize=False)(torch.from_numpy(synth_waveform(5000, 3, 5000)).to(cuda))
    # near-denormal amplitudes: squares of 1e-21 samples are f32 denormals, Parseval only holds to the floors
    tiny = synth_waveform(9, 3, 20_000) * np.array([[1e-19], [1e-21], [1e-23]], np.float32)
    t_out = GpuLogMel(normalize=False)(torch.from_numpy(tiny).to(cuda)).cpu().numpy()
    np.testing.assert_allclose(t_out, olog.logmel(tiny, normalize=False).numpy(), atol=ATOL, rtol=0)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert w.cpu().tolist() == [0] * 8


def test_self_check_passes_non_finite_clips(cuda, monkeypatch):
    """A NaN or Inf sample corrupts its own clip (as in the reference) without reading as a failed transform, and
    the clean clip beside it is unchanged."""
    w = _fresh_err_word(monkeypatch, cuda)
    wav = synth_waveform(13, 3, 20_000)
    mel = GpuLogMel(normalize=False)
    clean = mel(torch.from_numpy(wav).to(cuda)).cpu().numpy()
    wav[1, 7000] = np.nan
    wav[2, 12000] = np.inf
    out = mel(torch.from_numpy(wav).to(cuda)).cpu().numpy()
    torch.cuda.synchronize()
    assert w.cpu().tolist() == [0] * 8
    np.testing.assert_array_equal(out[0], clean[0])
    assert (out[1] != clean[1]).any() and (out[2] != clean[2]).any()


def test_self_check_repairs_a_transient_fault(cuda, monkeypatch):
    """One spectrum value of clip 1, frame 293 scaled by 1.05 on the first attempt only (MIA_LOGMEL_FAULT): the
    check catches it, the frame is recomputed, the output is bit-identical to a clean call, and err[4..7] record
    (clip 1 + 1, frame 293, wave 1) -- frame 293 is item 18's frame 5, i.e. wave 1's."""
    from src.miaudio import kernels as K
    wav = torch.from_numpy(synth_waveform(71, 2, 220_500)).to(cuda)
    mel = GpuLogMel()
    clean = mel(wav).clone()
    w = _fresh_err_word(monkeypatch, cuda)
    monkeypatch.setenv("MIA_LOGMEL_FAULT", "1,293,1")
    again = mel(wav)
    torch.cuda.synchronize()
    assert w.cpu().tolist() == [0, 0, 0, 0, 1, 2, 293, 1]
    assert torch.equal(again, clean)
    K.check_logmel_errors()  # a repaired frame is not an error


def test_self_check_flags_a_persistent_fault(cuda, monkeypatch):
    """The same fault on every attempt: err[0..3] record it and check_logmel_errors raises; only that clip differs."""
    from src.miaudio import kernels as K
    wav = torch.from_numpy(synth_waveform(71, 2, 220_500)).to(cuda)
    mel = GpuLogMel(normalize=False)
    clean = mel(wav).clone()
    w = _fresh_err_word(monkeypatch, cuda)
    monkeypatch.setenv("MIA_LOGMEL_FAULT", "1,293,3")
    bad = mel(wav)
    torch.cuda.synchronize()
    assert w.cpu().tolist() == [1, 2, 293, 1, 0, 0, 0, 0]
    diff = (bad != clean).nonzero()
    assert diff.shape[0] > 0 and set(diff[:, 0].tolist()) == {1} and set(diff[:, 2].tolist()) == {293}
    with pytest.raises(RuntimeError, match="clip 1, frame 293, wave 1"):
        K.check_logmel_errors()
