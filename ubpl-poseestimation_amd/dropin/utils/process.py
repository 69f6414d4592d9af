"""utils/process.py: the hot-path methods of ProcessUtils on the HIP path; with
UBPL_REFERENCE_ROOT set, every other method (image I/O, resize, drawing, ...)
is inherited from the reference's own class."""
import importlib.util
import os

from ubpl_amd.process import ProcessUtils as _Hot

_base = object
_ref = os.environ.get("UBPL_REFERENCE_ROOT")
if _ref and os.path.exists(os.path.join(_ref, "utils", "process.py")):
    _spec = importlib.util.spec_from_file_location("utils._reference_process", os.path.join(_ref, "utils", "process.py"),
                                                   submodule_search_locations=None)
    _mod = importlib.util.module_from_spec(_spec)
    _mod.__package__ = "utils"
    _spec.loader.exec_module(_mod)
    _base = _mod.ProcessUtils


class ProcessUtils(_Hot, _base):
    pass
