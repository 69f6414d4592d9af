from ubpl_amd.hourglass import StackedHourglass  # noqa: F401
