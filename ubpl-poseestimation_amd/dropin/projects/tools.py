"""projects/tools.py: ProjectTools."""
from ubpl_amd.tools import ProjectTools  # noqa: F401
