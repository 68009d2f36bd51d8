from voiceactivityprojection_amd.model import (  # noqa: F401
    BIN_TIMES, VAPModel, VapConfig, VapGPT, VapGPTMono, VapMonoConfig, load_older_state_dict)
from voiceactivityprojection_amd.utils import everything_deterministic, vad_fill_silences, vad_omit_spikes  # noqa: F401
