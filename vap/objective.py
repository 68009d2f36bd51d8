from voiceactivityprojection_amd.objective import (  # noqa: F401
    Codebook, ObjectiveVAP, ProjectionWindow, bin_times_to_frames)
