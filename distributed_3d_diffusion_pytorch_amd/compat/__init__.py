from .diff3d import Diff3D

__all__ = ["Diff3D"]
