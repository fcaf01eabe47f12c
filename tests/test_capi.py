"""CPU: the C-ABI library loads, exports exactly what include/dexiraft_corr.h
declares, and validates arguments on the host before any launch (so these calls
are safe without a GPU: they return before touching the device)."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from conftest import REPO

HEADER = REPO / "include" / "dexiraft_corr.h"
DECL = re.compile(r"^\s*(?:int|int64_t|const char\*)\s+(dxr_\w+)\s*\(", re.M)


def declared() -> set[str]:
    return set(DECL.findall(HEADER.read_text()))


@pytest.fixture(scope="module")
def nat():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_dxr_build_t", REPO / "optical-flow_dexi-raft_amd" / "build.py")
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    b.build()  # no-op when fresh; hipcc cross-compiles here otherwise
    from dexiraft_amd import _native
    _native.load()
    return _native


def test_header_declares_the_documented_entry_points():
    assert declared() == {
        "dxr_abi_version", "dxr_status_string", "dxr_last_hip_error", "dxr_pyramid_numel",
        "dxr_pyramid_level_offset", "dxr_corr_pyramid_build", "dxr_corr_lookup",
        "dxr_build_workspace_bytes", "dxr_corr_pyramid_build_ws",
        "dxr_avg_pool2x2", "dxr_alt_corr_forward", "dxr_alt_corr_lookup", "dxr_corr_volume",
        "dxr_pyramid_unpack", "dxr_pyramid_pack",
        "dxr_corr_lookup_backward", "dxr_pyramid_backward", "dxr_alt_corr_backward",
        "dxr_conv1x1_packed_bytes", "dxr_conv1x1_pack_weight", "dxr_corr_lookup_conv1x1",
        "dxr_transpose", "dxr_avg_pool2x2_nhwc", "dxr_alt_workspace_bytes",
        "dxr_alt_corr_lookup_ws", "dxr_fmap_grads_workspace_bytes", "dxr_fmap_grads",
        "dxr_corr_lookup_backward_multi", "dxr_lookup_backward_bound_slots",
        "dxr_corr_lookup_backward_multi_bound", "dxr_fmap_grads_bounded",
        "dxr_fmap_grads_bounded_workspace_bytes", "dxr_alt_corr_lookup_levels_ws",
        "dxr_alt_volume_numel", "dxr_alt_coarse_volumes", "dxr_alt_volume_lookup",
        "dxr_alt_coarse_volumes_ws_bytes", "dxr_alt_coarse_volumes_ws"}


def test_library_exports_every_declared_symbol(nat):
    out = subprocess.run(["nm", "-D", "--defined-only", str(nat.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T dxr_" in ln}
    assert exported == declared()
    assert set(nat.SIGNATURES) == declared()
    lib = nat.load()
    for name in declared():
        assert isinstance(getattr(lib, name), ctypes._CFuncPtr)


def test_library_is_gfx950_code(nat):
    """The embedded HIP fat binary targets gfx950 (MI355X) only."""
    blob = Path(nat.LIB_PATH).read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_abi_version_and_status_strings(nat):
    lib = nat.load()
    assert lib.dxr_abi_version() == nat.ABI_VERSION == 10
    assert lib.dxr_status_string(0) == b"ok"
    assert lib.dxr_status_string(1) == b"invalid argument"
    assert lib.dxr_status_string(2) == b"unsupported by this build"
    assert lib.dxr_status_string(-1) == b"HIP launch error"
    assert lib.dxr_status_string(77) == b"unknown status"
    assert lib.dxr_last_hip_error() == 0


@pytest.mark.parametrize("B,H,W,L", [(1, 55, 128, 4), (8, 47, 156, 4), (2, 12, 16, 4),
                                     (1, 33, 40, 5), (3, 9, 11, 2), (1, 1, 1, 1)])
def test_pyramid_geometry(nat, B, H, W, L):
    """Paged sizes: levels 0..3 in pages of 128 queries x (8x16 >> l) cells over
    whole tiles; levels >= 4 row-major (include/dexiraft_corr.h)."""
    lib = nat.load()
    n = H * W
    qt, ty, tx = -(-n // 128), -(-H // 8), -(-W // 16)
    offs = [0]
    h, w = H, W
    for lvl in range(L):
        if lvl:
            h, w = h // 2, w // 2
        if lvl < 4:
            offs.append(offs[-1] + B * qt * 128 * ty * tx * (8 >> lvl) * (16 >> lvl))
        else:
            offs.append(offs[-1] + B * n * h * w)
    assert lib.dxr_pyramid_numel(B, H, W, L) == offs[-1]
    for lvl in range(L):
        assert lib.dxr_pyramid_level_offset(B, H, W, lvl) == offs[lvl]


def test_pyramid_geometry_rejects_empty_levels(nat):
    lib = nat.load()
    assert lib.dxr_pyramid_numel(1, 7, 30, 4) == -1     # 7 -> 3 -> 1 -> 0
    assert lib.dxr_pyramid_numel(1, 8, 8, 4) > 0
    assert lib.dxr_pyramid_numel(1, 8, 8, 0) == -1
    assert lib.dxr_pyramid_level_offset(1, 8, 8, -1) == -1


def test_host_side_validation_needs_no_gpu(nat):
    lib = nat.load()
    P = 1 << 12  # a non-null dummy address: never dereferenced on these paths
    EINVAL, EUNSUP, OK = nat.DXR_EINVAL, nat.DXR_EUNSUPPORTED, nat.DXR_OK
    b = lib.dxr_corr_pyramid_build
    # (fmap1, fmap2, in_dtype, layout, B, D, H, W, L, divisor, pyramid, pyr_dtype, algo, stream)
    assert b(P, P, 0, 0, -1, 256, 8, 8, 4, 16.0, P, 0, 0, None) == EINVAL      # B < 0
    assert b(P, P, 0, 0, 1, 0, 8, 8, 4, 16.0, P, 0, 0, None) == EINVAL        # D = 0
    assert b(P, P, 0, 0, 1, 256, 7, 30, 4, 16.0, P, 0, 0, None) == EINVAL     # empty level
    assert b(P, P, 0, 0, 1, 256, 8, 8, 4, 0.0, P, 0, 0, None) == EINVAL       # divisor 0
    assert b(P, P, 0, 0, 1, 256, 8, 8, 4, float("nan"), P, 0, 0, None) == EINVAL
    assert b(None, P, 0, 0, 1, 256, 8, 8, 4, 16.0, P, 0, 0, None) == EINVAL   # null input
    assert b(P, P, 0, 0, 0, 256, 8, 8, 4, 16.0, None, 0, 0, None) == OK       # empty batch
    assert b(P, P, 7, 0, 1, 256, 8, 8, 4, 16.0, P, 0, 0, None) == EINVAL      # unknown dtype
    assert b(P, P, 0, 2, 1, 256, 8, 8, 4, 16.0, P, 0, 0, None) == EINVAL      # unknown layout
    assert b(P, P, 0, 0, 1, 256, 8, 8, 4, 16.0, P, 0, 9, None) == EINVAL      # unknown algo
    assert b(P, P, 1, 0, 1, 256, 8, 8, 4, 16.0, P, 1, 1, None) == EUNSUP      # exact-f32 of bf16
    # bf16 pyramid beyond the four fused levels: refused before any launch
    assert b(P, P, 1, 0, 1, 256, 64, 64, 5, 16.0, P, 1, 0, None) == EUNSUP
    assert lib.dxr_corr_volume(P, P, 0, 1, 0, 8, 8, 16.0, P, None) == EINVAL
    assert lib.dxr_pyramid_unpack(P, 0, 1, 8, 8, 4, 4, P, None) == EINVAL   # level >= L
    assert lib.dxr_pyramid_pack(P, 1, 8, 8, 4, 0, P, 3, None) == EINVAL     # bad dtype
    lk = lib.dxr_corr_lookup
    assert lk(P, 0, 1, 8, 8, 4, -1, P, P, None) == EINVAL               # radius < 0
    assert lk(P, 0, 1, 8, 8, 4, 9, P, P, None) == EUNSUP                # radius > 8
    assert lk(P, 0, 1, 8, 8, 9, 4, P, P, None) == EINVAL                # 9 levels
    assert lk(P, 5, 1, 8, 8, 4, 4, P, P, None) == EINVAL                # unknown dtype
    assert lk(P, 0, 0, 8, 8, 4, 4, None, None, None) == OK
    assert lk(P, 0, 1, 8, 8, 4, 4, None, P, None) == EINVAL             # null coords
    assert lib.dxr_avg_pool2x2(P, P, -1, 8, 8, None) == EINVAL
    assert lib.dxr_avg_pool2x2(None, None, 0, 8, 8, None) == OK
    assert lib.dxr_avg_pool2x2(P, P, 3, 1, 8, None) == OK               # nothing to pool
    tr = lib.dxr_transpose
    assert tr(P, P, 2, 1, 8, 8, None) == EINVAL                         # unknown dtype
    assert tr(P, P, 0, -1, 8, 8, None) == EINVAL
    assert tr(None, None, 0, 1, 0, 8, None) == OK                       # empty
    assert tr(None, P, 1, 1, 8, 8, None) == EINVAL                      # null input
    pn = lib.dxr_avg_pool2x2_nhwc
    assert pn(P, P, 1, 8, 8, 0, None) == EINVAL                         # no channels
    assert pn(None, None, 1, 1, 8, 64, None) == OK                      # nothing to pool
    assert pn(None, P, 1, 8, 8, 64, None) == EINVAL
    af = lib.dxr_alt_corr_forward
    assert af(P, P, P, P, 1, 8, 8, 8, 8, 64, 1, -1, None) == EINVAL
    assert af(P, P, P, P, 1, 8, 8, 8, 8, 64, 1, 7, None) == EUNSUP
    assert af(P, P, P, P, 1, 8, 8, 8, 8, 0, 1, 4, None) == EINVAL
    assert af(None, None, None, None, 1, 8, 8, 8, 8, 64, 0, 4, None) == OK
    al = lib.dxr_alt_corr_lookup
    ptrs = (ctypes.c_void_p * 4)(P, P, P, P)
    assert al(P, ptrs, P, P, 1, 16, 16, 64, 4, 4, 0.0, None) == EINVAL  # divisor 0
    assert al(P, ptrs, P, P, 1, 16, 16, 64, 4, 9, 16.0, None) == EUNSUP
    assert al(P, None, P, P, 1, 16, 16, 64, 4, 4, 16.0, None) == EINVAL
    lb = lib.dxr_corr_lookup_backward
    assert lb(P, P, 1, 8, 8, 4, -1, P, 0, None) == EINVAL               # radius < 0
    assert lb(P, P, 1, 8, 8, 4, 4, P, 1, None) == EUNSUP                # bf16 gradients
    assert lb(None, P, 1, 8, 8, 4, 4, P, 0, None) == EINVAL             # null coords
    assert lb(None, None, 0, 8, 8, 4, 4, None, 0, None) == OK           # empty batch
    ab = lib.dxr_alt_corr_backward
    assert ab(P, P, P, P, P, P, 1, 8, 8, 8, 8, 64, 1, -1, None) == EINVAL   # radius < 0
    assert ab(P, P, P, P, P, P, 1, 8, 8, 8, 8, 64, 1, 7, None) == EUNSUP    # radius > 6
    assert ab(P, P, P, P, P, P, 1, 8, 8, 8, 8, 0, 1, 4, None) == EINVAL     # C = 0
    assert ab(P, P, None, P, P, P, 1, 8, 8, 8, 8, 64, 1, 4, None) == EINVAL  # null coords
    assert ab(P, P, P, P, None, P, 1, 8, 8, 8, 8, 64, 1, 4, None) == EINVAL  # null fmap1_grad
    assert ab(None, None, None, None, None, None, 0, 8, 8, 8, 8, 64, 1, 4, None) == OK
    assert lib.dxr_conv1x1_packed_bytes(256, 324) == 336 * 256 * 4 * 2   # f32 + f16-pair copies
    assert lib.dxr_conv1x1_packed_bytes(0, 324) == -1
    assert lib.dxr_conv1x1_pack_weight(P, 0, 324, P, None) == EINVAL
    assert lib.dxr_conv1x1_pack_weight(None, 256, 324, P, None) == EINVAL
    lc = lib.dxr_corr_lookup_conv1x1
    assert lc(P, 0, 1, 8, 8, 4, -1, P, P, P, 256, 1, P, None) == EINVAL     # radius < 0
    assert lc(P, 0, 1, 8, 8, 4, 2, P, P, P, 256, 1, P, None) == EUNSUP     # radius 2
    assert lc(P, 0, 1, 8, 8, 4, 4, P, P, P, 100, 1, P, None) == EUNSUP     # Cout % 32
    assert lc(P, 0, 1, 64, 64, 5, 4, P, P, P, 256, 1, P, None) == EUNSUP   # 5 levels
    assert lc(P, 0, 1, 8, 8, 4, 4, P, None, P, 256, 1, P, None) == EINVAL  # null weights
    assert lc(P, 7, 1, 8, 8, 4, 4, P, P, P, 256, 1, P, None) == EINVAL     # unknown dtype
    assert lc(None, 0, 0, 8, 8, 4, 4, None, None, None, 256, 1, None, None) == OK
    pb = lib.dxr_pyramid_backward
    assert pb(P, 0, 1, 8, 8, 4, 0.0, P, None) == EINVAL                 # divisor 0
    assert pb(P, 0, 1, 7, 30, 4, 16.0, P, None) == EINVAL               # empty level
    assert pb(P, 1, 1, 8, 8, 4, 16.0, P, None) == EUNSUP
    assert lib.dxr_last_hip_error() == 0


def test_check_maps_status_to_reference_exceptions(nat):
    nat.check(0, "ok")
    with pytest.raises(RuntimeError, match="invalid argument"):
        nat.check(1, "x")
    with pytest.raises(NotImplementedError):
        nat.check(2, "x")


def test_build_workspace_bytes(nat):
    """The pre-split f32 build's workspace (ABI 6): two f16-pair operand copies
    (4 B per f32 element) and two int32 exponents per pixel, each 256-B aligned;
    bf16 fmaps with D % 32 == 0 the pack pass's two blocked copies; other D
    need none; bad geometry is -1."""
    lib = nat.load()
    al = lambda x: (x + 255) // 256 * 256   # noqa: E731
    for B, D, H, W in ((1, 256, 55, 128), (8, 256, 47, 156), (2, 64, 13, 19)):
        N = H * W
        assert lib.dxr_build_workspace_bytes(nat.DXR_F32, B, D, H, W) == \
            2 * al(B * D * N * 4) + 2 * al(B * N * 4)
    # bf16: the pack pass's blocked copies of both fmaps (2 B per element)
    assert lib.dxr_build_workspace_bytes(nat.DXR_BF16, 1, 256, 55, 128) == 2 * al(256 * 7040 * 2)
    assert lib.dxr_build_workspace_bytes(nat.DXR_BF16, 1, 48, 55, 128) == 0
    assert lib.dxr_build_workspace_bytes(nat.DXR_F32, 1, 24, 55, 128) == 0
    assert lib.dxr_build_workspace_bytes(nat.DXR_F32, -1, 256, 55, 128) == -1
    P = 1 << 12
    bw = lib.dxr_corr_pyramid_build_ws
    # validation is the plain build's: same statuses before any launch
    assert bw(P, P, 0, 0, 1, 0, 8, 8, 4, 16.0, P, 0, 0, P, 1 << 20, None) == nat.DXR_EINVAL
    assert bw(P, P, 0, 0, 0, 256, 8, 8, 4, 16.0, None, 0, 0, None, 0, None) == nat.DXR_OK


def test_alt_workspace_bytes(nat):
    """The on-the-fly lookup's query-order workspace, per level and coordinate
    set: a 16-byte entry and a bin id per query slot of every 4 x 8 query tile,
    64 blocks' histograms of 4097 bins, the bins' totals and the blocks' box
    costs, 16-byte aligned."""
    lib = nat.load()
    for B, H, W, L in ((1, 136, 240, 4), (2, 55, 128, 4), (3, 17, 19, 2)):
        np_ = -(-H // 4) * -(-W // 8) * 32
        per_list = (20 * np_ + 4 * 64 * 4097 + 4 * 4097 + 4 * 64 + 15) // 16 * 16
        assert lib.dxr_alt_workspace_bytes(B, H, W, L) == B * L * per_list
    assert lib.dxr_alt_workspace_bytes(1, 0, 8, 4) == -1
    assert lib.dxr_alt_workspace_bytes(1, 8, 8, 9) == -1
    P = 1 << 12
    aw = lib.dxr_alt_corr_lookup_ws
    ptrs = (ctypes.c_void_p * 4)(P, P, P, P)
    # validation as the workspace-less entry point, before any launch
    assert aw(P, ptrs, P, P, 1, 16, 16, 64, 4, 4, 0.0, P, 1 << 20, None) == nat.DXR_EINVAL
    assert aw(P, ptrs, P, P, 1, 16, 16, 64, 4, 9, 16.0, P, 1 << 20, None) == nat.DXR_EUNSUPPORTED
    assert aw(None, None, None, None, 0, 16, 16, 64, 4, 4, 16.0, None, 0, None) == nat.DXR_OK


def test_alt_coarse_volume_sizes(nat):
    """The coarse-level volumes: dxr_alt_volume_numel floats = the tail of a
    num_levels-level paged pyramid from first_level on; the volume GEMM's
    LDS-DMA workspace (dxr_alt_coarse_volumes_ws_bytes) = fmap1's and each tiled
    level's f16 pair planes (4 B per element, 256-B aligned regions), 0 when no
    level takes the GEMM (C % 32 != 0, or only row-major levels), -1 for bad
    geometry; the entry points validate before any launch."""
    lib = nat.load()
    al = lambda x: (x + 255) // 256 * 256   # noqa: E731
    for B, H, W, L, first in ((1, 136, 240, 4, 2), (2, 55, 128, 4, 1), (1, 48, 70, 5, 3)):
        assert lib.dxr_alt_volume_numel(B, H, W, L, first) == \
            lib.dxr_pyramid_numel(B, H, W, L) - lib.dxr_pyramid_numel(B, H, W, first)
        sizes, h, w = [], H, W
        for lvl in range(L):
            sizes.append((h, w))
            h, w = h // 2, w // 2
        want = al(B * H * W * 256 * 4) + sum(al(B * sizes[lvl][0] * sizes[lvl][1] * 256 * 4)
                                               for lvl in range(first, min(L, 4)))
        assert lib.dxr_alt_coarse_volumes_ws_bytes(B, H, W, 256, L, first) == want
    assert lib.dxr_alt_coarse_volumes_ws_bytes(1, 48, 70, 48, 4, 2) == 0     # C % 32
    assert lib.dxr_alt_coarse_volumes_ws_bytes(1, 48, 70, 64, 5, 4) == 0     # row-major only
    assert lib.dxr_alt_coarse_volumes_ws_bytes(1, 48, 70, 64, 4, 4) == -1    # first >= levels
    assert lib.dxr_alt_volume_numel(1, 48, 70, 4, 0) == lib.dxr_pyramid_numel(1, 48, 70, 4)
    assert lib.dxr_alt_volume_numel(1, 0, 70, 4, 1) == -1
    P = 1 << 12
    ptrs = (ctypes.c_void_p * 4)(P, P, P, P)
    cv, cvw = lib.dxr_alt_coarse_volumes, lib.dxr_alt_coarse_volumes_ws
    assert cv(P, ptrs, 1, 48, 70, 64, 4, 4, P, None) == nat.DXR_EINVAL          # first level
    assert cv(P, ptrs, 1, 48, 70, 40, 4, 2, P, None) == nat.DXR_EUNSUPPORTED    # C % 16
    assert cvw(P, ptrs, 1, 48, 70, 64, 4, 0, None, None, 0, None) == nat.DXR_EINVAL  # no volumes
    assert cv(None, None, 0, 48, 70, 64, 4, 2, None, None) == nat.DXR_OK       # B = 0


def _fmap_grads_ws(B, D, H, W):
    """dxr_fmap_grads' workspace: the larger of its two GEMMs' needs, each the
    three-way split fmap operand (3 x 16 bit per element, k padded to whole
    k-blocks of 128) plus, when K is split into S > 1 chunks (~256 workgroups),
    S - 1 partial [B, D, H*W] f32 sums (chunk 0 sums into the output itself)."""
    al = lambda x: (x + 255) // 256 * 256   # noqa: E731
    N = H * W
    qt, tiles = -(-N // 128), -(-H // 8) * -(-W // 16)
    slabs = -(-D // 256)
    need = 0
    for nblk, kbt in ((qt, tiles), (tiles, qt)):
        units = nblk * B * slabs
        S = 1 if units >= 256 else min(256 // units, kbt)
        op = al(B * 3 * kbt * 8 * D * 32)
        need = max(need, op + (al((S - 1) * B * D * N * 4) if S > 1 else 0))
    return need


def test_fmap_grads_workspace_and_validation(nat):
    lib = nat.load()
    for B, D, H, W in ((1, 256, 55, 128), (2, 64, 23, 37), (8, 256, 47, 156), (1, 288, 46, 62)):
        assert lib.dxr_fmap_grads_workspace_bytes(B, D, H, W, 4) == _fmap_grads_ws(B, D, H, W)
    assert lib.dxr_fmap_grads_workspace_bytes(1, 48, 55, 128, 4) == -1   # D % 32
    assert lib.dxr_fmap_grads_workspace_bytes(1, 256, 55, 128, 5) == -1  # row-major level
    assert lib.dxr_fmap_grads_workspace_bytes(1, 256, 0, 128, 4) == -1
    P = 1 << 12
    fg = lib.dxr_fmap_grads
    ws = _fmap_grads_ws(1, 256, 16, 16)
    # statuses before any launch
    assert fg(P, 0, P, P, 1, 256, 16, 16, 4, 0.0, P, P, P, ws, None) == nat.DXR_EINVAL
    assert fg(P, 1, P, P, 1, 256, 16, 16, 4, 16.0, P, P, P, ws, None) == nat.DXR_EUNSUPPORTED
    assert fg(P, 0, P, P, 1, 48, 16, 16, 4, 16.0, P, P, P, ws, None) == nat.DXR_EUNSUPPORTED
    assert fg(P, 0, P, P, 1, 256, 16, 16, 5, 16.0, P, P, P, ws, None) == nat.DXR_EUNSUPPORTED
    assert fg(P, 0, P, P, 1, 256, 16, 16, 4, 16.0, P, P, P, ws - 1, None) == nat.DXR_EINVAL
    assert fg(P, 0, P, P, 1, 256, 16, 16, 4, 16.0, P, P, None, ws, None) == nat.DXR_EINVAL
    assert fg(None, 0, None, None, 0, 256, 16, 16, 4, 16.0, None, None, None, 0, None) == nat.DXR_OK
    assert fg(P, 0, P, P, 1, 256, 16, 16, 4, 16.0, None, None, None, 0, None) == nat.DXR_OK


def test_lookup_backward_multi_validation(nat):
    lib = nat.load()
    P = 1 << 12
    arr = (ctypes.c_void_p * 17)(*([P] * 17))
    fn = lib.dxr_corr_lookup_backward_multi
    assert fn(arr, arr, 17, 1, 16, 16, 4, 4, P, nat.DXR_F32, None) == nat.DXR_EUNSUPPORTED
    assert fn(arr, arr, -1, 1, 16, 16, 4, 4, P, nat.DXR_F32, None) == nat.DXR_EINVAL
    assert fn(arr, arr, 2, 1, 16, 16, 4, 9, P, nat.DXR_F32, None) == nat.DXR_EUNSUPPORTED
    assert fn(arr, arr, 2, 1, 16, 16, 4, 4, None, nat.DXR_F32, None) == nat.DXR_EINVAL
    nul = (ctypes.c_void_p * 2)(P, None)
    assert fn(arr, nul, 2, 1, 16, 16, 4, 4, P, nat.DXR_F32, None) == nat.DXR_EINVAL
    assert fn(None, None, 0, 1, 16, 16, 4, 4, P, nat.DXR_F32, None) == nat.DXR_OK
    assert fn(arr, arr, 2, 0, 16, 16, 4, 4, P, nat.DXR_F32, None) == nat.DXR_OK


def test_bounded_backward_entry_points_validation(nat):
    lib = nat.load()
    P = 1 << 12
    # one slot per lookup-backward workgroup: 32 (r = 4) queries x level x pair
    for B, H, W, L, r in ((1, 55, 128, 4, 4), (2, 23, 37, 3, 3), (1, 16, 16, 4, 8)):
        n = lib.dxr_lookup_backward_bound_slots(B, H, W, L, r)
        assert n > 0 and n % (L * B) == 0 and (n // (L * B)) * 64 >= H * W
    assert lib.dxr_lookup_backward_bound_slots(1, 16, 16, 4, 9) == -1
    assert lib.dxr_lookup_backward_bound_slots(1, 0, 16, 4, 4) == -1
    arr = (ctypes.c_void_p * 17)(*([P] * 17))
    fb = lib.dxr_corr_lookup_backward_multi_bound
    assert fb(arr, arr, 2, 1, 16, 16, 4, 4, P, nat.DXR_F32, None, None) == nat.DXR_EINVAL  # no slots
    assert fb(arr, arr, 17, 1, 16, 16, 4, 4, P, nat.DXR_F32, P, None) == nat.DXR_EUNSUPPORTED
    assert fb(arr, arr, 2, 1, 16, 16, 4, 9, P, nat.DXR_F32, P, None) == nat.DXR_EUNSUPPORTED
    assert fb(arr, arr, 2, 0, 16, 16, 4, 4, P, nat.DXR_F32, P, None) == nat.DXR_OK
    fg = lib.dxr_fmap_grads_bounded
    bw = lib.dxr_fmap_grads_bounded_workspace_bytes
    for B, D, H, W in ((1, 256, 55, 128), (2, 64, 23, 37), (8, 256, 47, 156), (1, 288, 46, 62)):
        assert 0 < bw(B, D, H, W, 4) < _fmap_grads_ws(B, D, H, W)
        assert lib.dxr_fmap_grads_workspace_bytes(B, D, H, W, 4) == _fmap_grads_ws(B, D, H, W)
    assert bw(1, 48, 55, 128, 4) == -1
    ws = bw(1, 256, 16, 16, 4)
    assert fg(P, 0, P, P, 1, 256, 16, 16, 4, 0.0, P, 1, P, P, P, ws, None) == nat.DXR_EINVAL
    assert fg(P, 1, P, P, 1, 256, 16, 16, 4, 16.0, P, 1, P, P, P, ws, None) == nat.DXR_EUNSUPPORTED
    assert fg(P, 0, P, P, 1, 48, 16, 16, 4, 16.0, P, 1, P, P, P, ws, None) == nat.DXR_EUNSUPPORTED
    assert fg(P, 0, P, P, 1, 256, 16, 16, 4, 16.0, None, 1, P, P, P, ws, None) == nat.DXR_EINVAL
    assert fg(P, 0, P, P, 1, 256, 16, 16, 4, 16.0, P, 0, P, P, P, ws, None) == nat.DXR_EINVAL
    assert fg(P, 0, P, P, 1, 256, 16, 16, 4, 16.0, P, 1, P, P, P, ws - 1, None) == nat.DXR_EINVAL
    assert fg(None, 0, None, None, 0, 256, 16, 16, 4, 16.0, None, 0, None, None, None, 0,
              None) == nat.DXR_OK
