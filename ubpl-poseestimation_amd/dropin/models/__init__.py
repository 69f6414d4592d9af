"""models (models/__init__.py:1-7): PoseModel on the HIP path."""
from ubpl_amd.hourglass import PoseModel, hg as HG  # noqa: F401

__all__ = ("PoseModel",)
