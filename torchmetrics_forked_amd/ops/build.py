"""Build the native library (HIP kernels for gfx950 + C++ host ops) in-tree with ``hipcc``.

No hipify, no ``torch.utils.cpp_extension`` CUDA path: every ``csrc/*.hip`` / ``csrc/*.cpp`` is compiled
directly with ``hipcc --offload-arch=gfx950`` into an object file (in parallel, skipped when up to date) and
linked into ``torchmetrics_forked_amd/ops/_tmx_native.so``.  Ops register themselves through
``TORCH_LIBRARY_FRAGMENT(tmx, ...)`` so Python reaches them as ``torch.ops.tmx.<name>`` (scriptable).

Usage: ``python -m torchmetrics_forked_amd.ops.build [-j N] [--force]``
"""
import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import List

PKG_DIR = Path(__file__).resolve().parents[1]
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD_DIR = REPO / "build" / "native"
LIB_PATH = PKG_DIR / "ops" / "_tmx_native.so"
ARCH = os.environ.get("TMX_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: cannot build the gfx950 native library")


def _torch_paths() -> List[str]:
    import torch

    root = Path(torch.__file__).resolve().parent
    return [str(root / "include"), str(root / "include" / "torch" / "csrc" / "api" / "include"), str(root / "lib")]


def _common_flags() -> List[str]:
    import torch

    abi = int(torch.compiled_with_cxx11_abi())
    inc, inc_api, _ = _torch_paths()
    return [
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"--offload-arch={ARCH}",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        f"-I{inc}",
        f"-I{inc_api}",
        f"-I{CSRC}",
    ]


def sources() -> List[Path]:
    return sorted([*CSRC.glob("*.hip"), *CSRC.glob("*.cpp")])


def _needs_build(src: Path, obj: Path) -> bool:
    if not obj.exists():
        return True
    deps = [src, *CSRC.glob("*.h")]
    return any(d.stat().st_mtime > obj.stat().st_mtime for d in deps)


def _compile(src: Path, force: bool) -> Path:
    obj = BUILD_DIR / (src.name + ".o")
    if not force and not _needs_build(src, obj):
        return obj
    cmd = [_hipcc(), *_common_flags(), "-c", str(src), "-o", str(obj)]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")
    return obj


def build(jobs: int = 8, force: bool = False, verbose: bool = True) -> Path:
    """Compile every native source for gfx950 and link ``_tmx_native.so``; returns the library path."""
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if not force and LIB_PATH.exists() and LIB_PATH.stat().st_mtime >= newest:
        if verbose:
            print(f"[tmx build] up to date: {LIB_PATH}")
        return LIB_PATH
    _, _, lib = _torch_paths()
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [
        _hipcc(),
        "-shared",
        "-fPIC",
        f"--offload-arch={ARCH}",
        *map(str, objs),
        f"-L{lib}",
        "-lc10",
        "-lc10_hip",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_hip",
        f"-Wl,-rpath,{lib}",
        "-o",
        str(tmp),
    ]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")
    os.replace(tmp, LIB_PATH)
    if verbose:
        print(f"[tmx build] built {LIB_PATH} from {len(srcs)} sources")
    return LIB_PATH


def main(argv: List[str] = sys.argv[1:]) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    build(jobs=args.jobs, force=args.force)


if __name__ == "__main__":
    main()
