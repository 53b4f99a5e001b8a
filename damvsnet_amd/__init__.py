"""damvsnet_amd — MI355X-native cascade-MVS cost-volume engine (drop-in for DAMVSNet's hot path).

Heavy imports (torch modules, the HIP library) are lazy so that ``damvsnet_amd.synth`` and
``damvsnet_amd.weights`` stay importable without a GPU or a built library.
"""

__all__ = ["CascadeMVSNet", "DepthNet", "homo_warping", "load_library"]


def __getattr__(name):
    if name in ("CascadeMVSNet",):
        from .cascade import CascadeMVSNet
        return CascadeMVSNet
    if name in ("DepthNet", "homo_warping"):
        from . import depthnet
        return getattr(depthnet, name)
    if name == "load_library":
        from ._capi import load_library
        return load_library
    raise AttributeError(name)
