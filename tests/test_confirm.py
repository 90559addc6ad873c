"""Level-3 confirm module (easywakeword_amd/confirm.py): front-end filters and the
batched Whisper-tiny path (random init offline: timing only, parity unpinned)."""
import numpy as np


def test_slaney_mel_matches_librosa_restatement():
    from easywakeword_amd.confirm import _slaney_mel
    from oracle.mfcc_ref import mel_filterbank
    np.testing.assert_allclose(_slaney_mel(16000, 512, 128), mel_filterbank(), rtol=2e-6, atol=1e-9)


def test_whisper_confirm_batch_runs_on_cpu():
    from easywakeword_amd.confirm import WhisperConfirm
    wc = WhisperConfirm(device="cpu", max_new_tokens=2)
    assert wc.random_init
    rng = np.random.default_rng(0)
    batch = [np.clip(rng.standard_normal(n) * 0.3, -1, 1) for n in (8000, 12000)]
    feats = wc.log_mel(batch)
    assert tuple(feats.shape) == (2, 80, 3000)
    out = wc.transcribe(batch)
    assert out == ["", ""]          # no tokenizer offline: empty text, i.e. never confirms
    assert wc(batch[0]) is None
