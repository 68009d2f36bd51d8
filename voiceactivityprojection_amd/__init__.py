"""MI355X-native VAP (Voice Activity Projection) inference engine.

Drop-in for the reference's ``vap.model`` API (see ``vap/`` shim package); compute runs in
hand-written HIP kernels for gfx950 behind the C ABI in include/vap_hip.h.
"""
from .model import BIN_TIMES, VAPModel, VapConfig, VapGPT, load_older_state_dict  # noqa: F401
from .objective import ObjectiveVAP  # noqa: F401

__version__ = "0.1.0"
