"""Register ``neural-collaborative-filtering-demo_amd/`` (not an identifier) as package ``ncf_amd``."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "neural-collaborative-filtering-demo_amd")


def load():
    if "ncf_amd" in sys.modules:
        return sys.modules["ncf_amd"]
    spec = importlib.util.spec_from_file_location(
        "ncf_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ncf_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
