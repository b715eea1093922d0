"""Register the `lamellar-runtime_amd/` directory as the importable package
`lamellar_runtime_amd` (a hyphen cannot appear in a Python module name)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "lamellar-runtime_amd")
PKG_NAME = "lamellar_runtime_amd"


def load_package():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except Exception:
        del sys.modules[PKG_NAME]
        raise
    return mod
