"""MI355X-native training path for NeuroSync Trainer Lite (audio -> ARKit blendshapes).

Module layout mirrors the reference (config, train, utils/*, dataset/*) so it is a
drop-in; compute runs in libnstl_hip.so (hand-written gfx950 HIP kernels).
"""
__version__ = "0.1.0"
