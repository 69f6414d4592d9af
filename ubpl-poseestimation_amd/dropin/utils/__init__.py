import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
import _ref  # noqa: E402

__path__ = _ref.extend(__path__, "utils")
