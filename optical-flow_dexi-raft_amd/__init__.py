"""dexiraft_amd — MI355X-native RAFT correlation subsystem (Dexi+RAFT hot path).

Import name ``dexiraft_amd`` (see ``dexiraft_amd.py`` at the repository root,
which maps it onto this ``optical-flow_dexi-raft_amd/`` directory).

Public surface, mirroring the reference's interface for this path:
  * ``CorrBlock``, ``AlternateCorrBlock``  — core/corr.py:12-91
  * ``alt_cuda_corr.forward / backward``  — alt_cuda_corr/correlation.cpp:51-54
  * ``coords_grid``                        — core/utils/utils.py:74-77
  * ``driver.InputPadder / write_flo / infer_pairs`` — core/utils/utils.py:7-24,
    core/utils/frame_utils.py:70-99, evaluate.py's per-pair loop (sharded)
"""
from . import alt_cuda_corr, driver
from ._native import LIB_PATH, load as load_native
from .corr import AlternateCorrBlock, CorrBlock
from .utils import coords_grid

__all__ = ["CorrBlock", "AlternateCorrBlock", "alt_cuda_corr", "coords_grid", "driver", "load_native",
           "LIB_PATH"]
__version__ = "0.1.0"
