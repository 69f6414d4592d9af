"""Locate the reference checkout for the modules outside the hot path."""
import os

REF = os.environ.get("UBPL_REFERENCE_ROOT")


def extend(pkg_path, *sub):
    """Append the reference's directory for this package to its __path__ so
    that out-of-scope submodules (e.g. utils.base) resolve to the reference."""
    if REF:
        d = os.path.join(REF, *sub)
        if os.path.isdir(d) and d not in pkg_path:
            pkg_path.append(d)
    return pkg_path
