"""models/pose/pose_model.py on the HIP path."""
from ubpl_amd.hourglass import pose_model  # noqa: F401
