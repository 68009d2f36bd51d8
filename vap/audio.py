from voiceactivityprojection_amd.audio import load_waveform, resample  # noqa: F401
from voiceactivityprojection_amd.utils import time_to_frames  # noqa: F401
