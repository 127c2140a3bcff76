"""Import shim: the package directory is `kafkastreams-cep_amd/` (not a Python identifier).

`import cepamd` loads it as the package `kafkastreams_cep_amd` and re-exports its API.
"""
import importlib.util as _u
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "kafkastreams-cep_amd")
if "kafkastreams_cep_amd" not in _sys.modules:
    _spec = _u.spec_from_file_location("kafkastreams_cep_amd", _os.path.join(_DIR, "__init__.py"),
                                       submodule_search_locations=[_DIR])
    _mod = _u.module_from_spec(_spec)
    _sys.modules["kafkastreams_cep_amd"] = _mod
    _spec.loader.exec_module(_mod)
from kafkastreams_cep_amd import *  # noqa: E402,F401,F403
from kafkastreams_cep_amd import __all__  # noqa: E402,F401
