"""Import alias: ``import dexiraft_amd`` loads the ``optical-flow_dexi-raft_amd/`` package.

The package directory name (required by the repository layout) is not a valid
Python identifier, so this module replaces itself in ``sys.modules`` with that
package (a supported pattern of the import system).
"""
import importlib.util
import sys
from pathlib import Path

_PKG_DIR = Path(__file__).resolve().parent / "optical-flow_dexi-raft_amd"
_spec = importlib.util.spec_from_file_location(
    __name__, _PKG_DIR / "__init__.py", submodule_search_locations=[str(_PKG_DIR)])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
