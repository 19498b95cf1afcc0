"""Import helper for the ``st-gcn_amd/`` package.

The package directory name contains a hyphen, so it cannot be imported by a
plain ``import`` statement; this registers it as the module ``stgcn_amd``.
"""
import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "st-gcn_amd")


def load():
    mod = sys.modules.get("stgcn_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "stgcn_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["stgcn_amd"] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop("stgcn_amd", None)
        raise
    return mod
