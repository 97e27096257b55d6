"""Import helper: the product package lives in the directory `mpir-fft_amd/`
(a name Python cannot import directly); this loads it as module `mpir_fft_amd`."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "mpir-fft_amd")


def load():
    mod = sys.modules.get("mpir_fft_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location("mpir_fft_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mpir_fft_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
