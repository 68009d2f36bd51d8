"""Drop-in namespace: ``from vap.model import VapGPT, VapConfig, VAPModel`` resolves to the MI355X
engine (voiceactivityprojection_amd)."""
