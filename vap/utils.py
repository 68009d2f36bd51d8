from voiceactivityprojection_amd.utils import *  # noqa: F401,F403
