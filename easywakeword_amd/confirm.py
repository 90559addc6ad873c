"""Level-3 confirm, batched on the GPU: Whisper-tiny in PyTorch-ROCm.

The reference transcribes each level-2 positive with openai-whisper
(``WakeWord._transcribe_audio``, wakeword.py:1009-1034, after the normalisation
that ``ewk_normalize_events`` runs on the device) and checks the text
(wakeword.py:1129-1153, ``WakeWord._check_transcription`` here).  This module
batches the gathered positives instead: Whisper's 80-bin log-mel front end on the
GPU (n_fft 400, hop 160, Slaney mel, log10, max-8 dB floor, 30 s window), then one
batched greedy decode of Whisper-tiny (``transformers.WhisperForConditionalGeneration``).

openai-whisper and its weights are not available offline: with ``weights=None``
the model is randomly initialised (timing only -- parity unpinned, the decoded
tokens are meaningless); pass a local Hugging Face checkpoint directory to get
real transcriptions.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np

SR = 16000
N_FFT = 400
HOP = 160
N_MELS = 80
N_FRAMES = 3000          # 30 s window


def _slaney_mel(sr: int, n_fft: int, n_mels: int) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels) (Slaney scale and norm) as float32 [n_mels, n_fft//2+1]."""
    f_sp = 200.0 / 3
    min_log_hz, logstep = 1000.0, math.log(6.4) / 27.0
    min_log_mel = min_log_hz / f_sp

    def hz_to_mel(f):
        f = np.asarray(f, np.float64)
        return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep, f / f_sp)

    def mel_to_hz(m):
        m = np.asarray(m, np.float64)
        return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)

    fft = np.linspace(0, sr / 2, n_fft // 2 + 1)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(0.0), hz_to_mel(sr / 2), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0.0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return w.astype(np.float32)


class WhisperConfirm:
    """Batched Whisper-tiny transcription of normalised segments on one GPU."""

    def __init__(self, device=None, weights: Optional[str] = None, max_new_tokens: int = 8):
        import torch
        from transformers import WhisperConfig, WhisperForConditionalGeneration
        self.torch = torch
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        if weights:
            self.model = WhisperForConditionalGeneration.from_pretrained(weights, local_files_only=True)
            self.random_init = False
            try:
                from transformers import WhisperProcessor
                self.processor = WhisperProcessor.from_pretrained(weights, local_files_only=True)
            except Exception:  # noqa: BLE001 - a checkpoint without tokenizer files still times
                self.processor = None
        else:
            torch.manual_seed(0)
            self.model = WhisperForConditionalGeneration(WhisperConfig())   # whisper-tiny dimensions
            self.random_init = True
            self.processor = None
        # bf16 on the GPU (MFMA), fp32 on the CPU
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.model = self.model.to(self.device, dtype=self.dtype).eval()
        self.max_new_tokens = max_new_tokens
        self.mel = torch.from_numpy(_slaney_mel(SR, N_FFT, N_MELS)).to(self.device)
        self.window = torch.hann_window(N_FFT, device=self.device)

    def log_mel(self, batch: Sequence[np.ndarray]):
        """Whisper's front end for a batch of 16 kHz segments -> [B, 80, 3000] float32."""
        torch = self.torch
        n = N_FRAMES * HOP
        x = torch.zeros((len(batch), n), dtype=torch.float32, device=self.device)
        for i, a in enumerate(batch):   # numpy arrays or device tensors (normalize_events_device)
            if torch.is_tensor(a):
                a = a[:n].to(device=self.device, dtype=torch.float32)
            else:
                a = torch.as_tensor(np.asarray(a, np.float32)[:n], device=self.device)
            x[i, :a.numel()] = a
        spec = torch.stft(x, N_FFT, HOP, window=self.window, return_complex=True)
        power = spec[..., :-1].abs() ** 2
        mel = self.mel @ power
        log_spec = torch.clamp(mel, min=1e-10).log10()
        log_spec = torch.maximum(log_spec, log_spec.amax(dim=(1, 2), keepdim=True) - 8.0)
        return (log_spec + 4.0) / 4.0

    def transcribe(self, batch: Sequence[np.ndarray]) -> List[str]:
        """Greedy transcription of each segment (empty strings for a random-init model)."""
        if not len(batch):
            return []
        torch = self.torch
        with torch.no_grad():
            feats = self.log_mel(batch).to(self.dtype)
            tokens = self.model.generate(input_features=feats, max_new_tokens=self.max_new_tokens,
                                         do_sample=False)
        if self.processor is not None:
            return list(self.processor.batch_decode(tokens, skip_special_tokens=True))
        return ["" for _ in range(len(batch))]

    def __call__(self, audio: np.ndarray) -> Optional[str]:
        """The WakeWord ``confirm`` callable: one normalised segment -> text."""
        return self.transcribe([audio])[0] or None
