"""Build libdexiraft_corr.so (HIP, gfx950) in-tree.

Every ``csrc/*.hip`` file is compiled with ``hipcc --offload-arch=gfx950`` into
``build/*.o`` and linked into ``libdexiraft_corr.so`` next to this file, so the
shared object travels with the repository snapshot to the GPU box.  No torch
headers are involved: the library is a plain C-ABI (include/dexiraft_corr.h).

Usage: ``python optical-flow_dexi-raft_amd/build.py [--force] [--asm]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC = PKG_DIR / "csrc"
INCLUDE = REPO_DIR / "include"
BUILD_DIR = PKG_DIR / "build"
LIB_NAME = "libdexiraft_corr.so"
LIB_PATH = PKG_DIR / LIB_NAME
# Experiments target (timing ablations; never loaded by the package): the
# csrc/experiments/*.hip files, each of which includes the product source it
# varies, objects in build/exp.
EXP_DIR = CSRC / "experiments"
EXP_LIB_PATH = PKG_DIR / "libdexiraft_corr_exp.so"
ARCH = "gfx950"

CXXFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-Wall", "-Wno-unused-function",
    f"-I{INCLUDE}", f"-I{CSRC}",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain (/opt/rocm) is required to build")


def _sources(experiments: bool = False) -> list[Path]:
    if experiments:   # each experiment includes its product source; capi.hip once
        return sorted(EXP_DIR.glob("*.hip")) + [CSRC / "capi.hip"]
    return sorted(CSRC.glob("*.hip"))


def _deps(experiments: bool = False) -> list[Path]:
    deps = _sources() + sorted(CSRC.glob("*.h")) + sorted(INCLUDE.glob("*.h")) + [Path(__file__)]
    return deps + (_sources(True) if experiments else [])


def is_stale(lib: Path = LIB_PATH) -> bool:
    if not lib.exists():
        return True
    t = lib.stat().st_mtime
    return any(p.stat().st_mtime > t for p in _deps(lib == EXP_LIB_PATH))


# Per-file flags.  corr_build.hip: no SLP vectorisation — packed f32 VALU
# (v_pk_add_f32) beside MFMAs costs more issue cycles than the scalar pair it
# replaces (MI355X_MICROARCH.md, cycle constants); measured r01: split build
# 192 -> 182 us at Sintel, other kernels neutral.
FILE_FLAGS = {"corr_build.hip": ["-fno-slp-vectorize"], "corr_lookup.hip": ["-fno-slp-vectorize"]}


def _compile(src: Path, extra: list[str], out_dir: Path = BUILD_DIR) -> Path:
    obj = out_dir / (src.stem + ".o")
    flags = FILE_FLAGS.get(src.name.replace("xp_", "corr_"), [])
    cmd = [hipcc(), *CXXFLAGS, *flags, *extra, "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{res.stderr}")
    if res.stderr.strip():
        sys.stderr.write(res.stderr)
    return obj


def build(force: bool = False, asm: bool = False, verbose: bool = False,
          experiments: bool = False) -> Path:
    """Compile and link the library if any source is newer than it
    (``experiments``: the separate timing-ablation target instead)."""
    lib = EXP_LIB_PATH if experiments else LIB_PATH
    if not force and not asm and not is_stale(lib):
        return lib
    out_dir = BUILD_DIR / "exp" if experiments else BUILD_DIR
    out_dir.mkdir(parents=True, exist_ok=True)
    extra = ["-save-temps=obj", "-Rpass-analysis=kernel-resource-usage"] if asm else []
    srcs = _sources(experiments)
    if not srcs:
        raise RuntimeError(f"no sources in {EXP_DIR if experiments else CSRC}")
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, extra, out_dir), srcs))
    tmp = lib.with_suffix(".so.tmp")
    cmd = [hipcc(), "-shared", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objs)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{res.stderr}")
    os.replace(tmp, lib)
    if verbose:
        print(f"built {lib}")
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asm", action="store_true", help="keep .s and print resource usage")
    ap.add_argument("--experiments", action="store_true",
                    help="build the timing-ablation target libdexiraft_corr_exp.so instead")
    a = ap.parse_args()
    build(force=a.force, asm=a.asm, verbose=True, experiments=a.experiments)
