"""models/pose/hourglass.py on the HIP path."""
from ubpl_amd.hourglass import StackedHourglass, hg  # noqa: F401
