"""neurecon_amd -- MI355X-native (gfx950) render path for neural-surface reconstruction
(NeuS / VolSDF / UNISURF), drop-in for SuwoongHeo/neurecon's model / volume_render API.

The compute lives in libnrhip.so (hand-written HIP for CDNA4, C-ABI in include/neurecon_hip.h);
this package mirrors the reference's Python interface on top of it.
"""
__version__ = '0.1.0'
