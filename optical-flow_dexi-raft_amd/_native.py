"""ctypes binding of libdexiraft_corr.so (C-ABI: include/dexiraft_corr.h).

The shared object is loaded only after ``import torch`` so that its
``libamdhip64.so.7`` dependency resolves to the HIP runtime torch already
loaded: device pointers and streams are then shared with torch's allocator.
There is no fallback: if the library is missing or a call fails, an exception
is raised.
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = Path(__file__).resolve().with_name("libdexiraft_corr.so")
ABI_VERSION = 10

DXR_OK, DXR_EINVAL, DXR_EUNSUPPORTED, DXR_EHIP = 0, 1, 2, -1
DXR_F32, DXR_BF16 = 0, 1
DXR_NCHW, DXR_NHWC = 0, 1
DXR_BUILD_AUTO, DXR_BUILD_EXACT_F32 = 0, 1

# Every symbol include/dexiraft_corr.h declares, with its ctypes signature.
_i64 = ctypes.c_int64
_int = ctypes.c_int
_vp = ctypes.c_void_p
_f32 = ctypes.c_float
SIGNATURES: dict[str, tuple[object, list[object]]] = {
    "dxr_abi_version": (_int, []),
    "dxr_status_string": (ctypes.c_char_p, [_int]),
    "dxr_last_hip_error": (_int, []),
    "dxr_pyramid_numel": (_i64, [_i64, _i64, _i64, _int]),
    "dxr_pyramid_level_offset": (_i64, [_i64, _i64, _i64, _int]),
    "dxr_corr_pyramid_build": (_int, [_vp, _vp, _int, _int, _i64, _i64, _i64, _i64, _int, _f32,
                                      _vp, _int, _int, _vp]),
    "dxr_build_workspace_bytes": (_i64, [_int, _i64, _i64, _i64, _i64]),
    "dxr_corr_pyramid_build_ws": (_int, [_vp, _vp, _int, _int, _i64, _i64, _i64, _i64, _int,
                                         _f32, _vp, _int, _int, _vp, _i64, _vp]),
    "dxr_corr_volume": (_int, [_vp, _vp, _int, _i64, _i64, _i64, _i64, _f32, _vp, _vp]),
    "dxr_pyramid_unpack": (_int, [_vp, _int, _i64, _i64, _i64, _int, _int, _vp, _vp]),
    "dxr_pyramid_pack": (_int, [_vp, _i64, _i64, _i64, _int, _int, _vp, _int, _vp]),
    "dxr_corr_lookup": (_int, [_vp, _int, _i64, _i64, _i64, _int, _int, _vp, _vp, _vp]),
    "dxr_avg_pool2x2": (_int, [_vp, _vp, _i64, _i64, _i64, _vp]),
    "dxr_corr_lookup_backward": (_int, [_vp, _vp, _i64, _i64, _i64, _int, _int, _vp, _int, _vp]),
    "dxr_corr_lookup_backward_multi": (_int, [ctypes.POINTER(_vp), ctypes.POINTER(_vp), _int, _i64,
                                              _i64, _i64, _int, _int, _vp, _int, _vp]),
    "dxr_lookup_backward_bound_slots": (_i64, [_i64, _i64, _i64, _int, _int]),
    "dxr_corr_lookup_backward_multi_bound": (_int, [ctypes.POINTER(_vp), ctypes.POINTER(_vp), _int,
                                                    _i64, _i64, _i64, _int, _int, _vp, _int, _vp,
                                                    _vp]),
    "dxr_pyramid_backward": (_int, [_vp, _int, _i64, _i64, _i64, _int, _f32, _vp, _vp]),
    "dxr_fmap_grads_workspace_bytes": (_i64, [_i64, _i64, _i64, _i64, _int]),
    "dxr_fmap_grads": (_int, [_vp, _int, _vp, _vp, _i64, _i64, _i64, _i64, _int, _f32, _vp, _vp,
                              _vp, _i64, _vp]),
    "dxr_fmap_grads_bounded_workspace_bytes": (_i64, [_i64, _i64, _i64, _i64, _int]),
    "dxr_fmap_grads_bounded": (_int, [_vp, _int, _vp, _vp, _i64, _i64, _i64, _i64, _int, _f32, _vp,
                                      _i64, _vp, _vp, _vp, _i64, _vp]),
    "dxr_alt_corr_forward": (_int, [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64,
                                    _i64, _int, _vp]),
    "dxr_alt_corr_backward": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64,
                                     _i64, _i64, _i64, _int, _vp]),
    "dxr_conv1x1_packed_bytes": (_i64, [_i64, _i64]),
    "dxr_conv1x1_pack_weight": (_int, [_vp, _i64, _i64, _vp, _vp]),
    "dxr_corr_lookup_conv1x1": (_int, [_vp, _int, _i64, _i64, _i64, _int, _int, _vp, _vp, _vp,
                                       _i64, _int, _vp, _vp]),
    "dxr_transpose": (_int, [_vp, _vp, _int, _i64, _i64, _i64, _vp]),
    "dxr_avg_pool2x2_nhwc": (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _vp]),
    "dxr_alt_corr_lookup": (_int, [_vp, ctypes.POINTER(_vp), _vp, _vp, _i64, _i64, _i64, _i64,
                                   _int, _int, _f32, _vp]),
    "dxr_alt_workspace_bytes": (_i64, [_i64, _i64, _i64, _int]),
    "dxr_alt_corr_lookup_ws": (_int, [_vp, ctypes.POINTER(_vp), _vp, _vp, _i64, _i64, _i64, _i64,
                                      _int, _int, _f32, _vp, _i64, _vp]),
    "dxr_alt_corr_lookup_levels_ws": (_int, [_vp, ctypes.POINTER(_vp), _vp, _vp, _i64, _i64, _i64,
                                             _i64, _int, _int, _int, _f32, _vp, _i64, _vp]),
    "dxr_alt_volume_numel": (_i64, [_i64, _i64, _i64, _int, _int]),
    "dxr_alt_coarse_volumes": (_int, [_vp, ctypes.POINTER(_vp), _i64, _i64, _i64, _i64, _int, _int,
                                      _vp, _vp]),
    "dxr_alt_coarse_volumes_ws_bytes": (_i64, [_i64, _i64, _i64, _i64, _int, _int]),
    "dxr_alt_coarse_volumes_ws": (_int, [_vp, ctypes.POINTER(_vp), _i64, _i64, _i64, _i64, _int,
                                         _int, _vp, _vp, _i64, _vp]),
    "dxr_alt_volume_lookup": (_int, [_vp, _vp, _vp, _i64, _i64, _i64, _int, _int, _int, _f32, _vp]),
}

_lock = threading.Lock()
_lib: ctypes.CDLL | None = None


def load() -> ctypes.CDLL:
    """Load (once) and return the native library; raise if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not LIB_PATH.exists():
                raise ImportError(
                    f"{LIB_PATH.name} not found next to {Path(__file__).name}; build it with "
                    "`python optical-flow_dexi-raft_amd/build.py` (hipcc, gfx950)")
            lib = ctypes.CDLL(str(LIB_PATH))
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            ver = lib.dxr_abi_version()
            if ver != ABI_VERSION:
                raise ImportError(f"{LIB_PATH.name} ABI {ver} != expected {ABI_VERSION}; rebuild")
            _lib = lib
    return _lib


def check(status: int, what: str) -> None:
    """Raise the exception the reference would raise for a failed call."""
    if status == DXR_OK:
        return
    lib = load()
    msg = lib.dxr_status_string(status).decode()
    if status == DXR_EHIP:
        raise RuntimeError(f"{what}: HIP error {lib.dxr_last_hip_error()} ({msg})")
    if status == DXR_EUNSUPPORTED:
        raise NotImplementedError(f"{what}: {msg}")
    raise RuntimeError(f"{what}: {msg}")


# torch's raw current-stream query: ~0.3 us per call against ~2 us for
# torch.cuda.current_stream(dev).cuda_stream, which builds a Stream object (the
# eager lookup path is host-bound: scripts/probe_host_overhead.py)
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t: torch.Tensor) -> int:
    """hipStream_t (as int) of torch's current stream on t's device."""
    if _raw_stream is not None:
        return _raw_stream(t.device.index)
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()
