"""Import shim: exposes the package directory `ai-laryngeal-video-based-classifier_amd/`
(whose name is not a Python identifier) as the importable package `vclip_amd`.

`import vclip_amd` replaces this module in sys.modules with the real package, so
`from vclip_amd.vivit import ...` resolves submodules inside that directory.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ai-laryngeal-video-based-classifier_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
