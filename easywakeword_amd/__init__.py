"""easywakeword_amd -- MI355X-native (gfx950) batched wake-word engine.

Drop-in for the hot path of raymondclowe/EasyWakeWord: the level-1 energy gate
(ring buffer + adaptive silence threshold + timing FSM) and the level-2
MFCC + cosine matcher, as hand-written HIP kernels behind a C ABI
(include/ewk.h, libewk.so) bound with ctypes.

    from easywakeword_amd import WakeWord, WordMatcher, StreamEngine
"""
from .engine import Engine, StreamEngine
from .wakeword import SoundBuffer, WakeWord, WordMatcher
from .audio import ArraySource, WavSource, load_wav, write_wav
from .devices import AudioDeviceManager

__all__ = ["WakeWord", "WordMatcher", "SoundBuffer", "Engine", "StreamEngine",
           "ArraySource", "WavSource", "load_wav", "write_wav", "AudioDeviceManager"]
__version__ = "0.1.0"
