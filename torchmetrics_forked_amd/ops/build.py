"""Build the native library (HIP kernels for gfx950 + C++ host ops) in-tree with ``hipcc``.

No hipify, no ``torch.utils.cpp_extension`` CUDA path: every ``csrc/*.hip`` / ``csrc/*.cpp`` is compiled
directly with ``hipcc --offload-arch=gfx950`` into an object file (in parallel) and linked into
``torchmetrics_forked_amd/ops/_tmx_native.so``.  Staleness is decided by CONTENT, not mtimes: each object is rebuilt
when the SHA-256 of its source + every header + the compile flags differs from the one recorded when it was built
(``build/native/manifest.json``), and the library is relinked when the digest of all sources differs from the stamp
``_tmx_native.so.sha256`` written next to it (that stamp travels with the library, so ``stale_sources()`` can tell
on any machine whether the ``.so`` matches the tree).  Ops register themselves through
``TORCH_LIBRARY_FRAGMENT(tmx, ...)`` so Python reaches them as ``torch.ops.tmx.<name>`` (scriptable).

Usage: ``python -m torchmetrics_forked_amd.ops.build [-j N] [--force]``
"""
import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import sysconfig
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


# per-source extra flags: image.hip's SSIM kernel keeps its MFMA accumulators in VGPRs (the AGPR form read every
# result back with one v_accvgpr_read per value: ~50 extra VALU instructions per band of its VALU-bound loop)
# py_columns.cpp is the library's CPython entry point (``ops.py_module()``): Python headers, libtorch_python at link
_EXTRA_FLAGS = {"image.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"], "py_columns.cpp": [f"-I{sysconfig.get_paths()['include']}"]}


def _flags_for(src: Path) -> List[str]:
    return [*_common_flags(), *_EXTRA_FLAGS.get(src.name, [])]


def sources() -> List[Path]:
    return sorted([*CSRC.glob("*.hip"), *CSRC.glob("*.cpp")])


MANIFEST = BUILD_DIR / "manifest.json"
STAMP = LIB_PATH.with_suffix(".so.sha256")


def _headers_digest() -> bytes:
    h = hashlib.sha256()
    for hdr in sorted(CSRC.glob("*.h")):
        h.update(hdr.name.encode())
        h.update(hdr.read_bytes())
    return h.digest()


def source_digest(src: Path, flags: List[str], headers: bytes) -> str:
    """SHA-256 of one translation unit's inputs: its text, every ``csrc`` header and the compile flags."""
    h = hashlib.sha256(src.read_bytes())
    h.update(headers)
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def tree_digest() -> str:
    """Digest of every native source and header (flags excluded: torch-independent, computable without hipcc)."""
    h = hashlib.sha256(_headers_digest())
    for src in sources():
        h.update(src.name.encode())
        h.update(src.read_bytes())
    return h.hexdigest()


def stale_sources() -> bool:
    """True when the in-tree library does not match the sources (missing, or built from other sources)."""
    if not LIB_PATH.exists() or not STAMP.exists() or not CSRC.exists():
        return not LIB_PATH.exists()
    return STAMP.read_text().strip() != tree_digest()


def _load_manifest() -> dict:
    try:
        return json.loads(MANIFEST.read_text())
    except Exception:
        return {}


def _compile(src: Path, digest: str, manifest: dict, force: bool) -> "tuple[Path, bool]":
    obj = BUILD_DIR / (src.name + ".o")
    if not force and obj.exists() and manifest.get(src.name) == digest:
        return obj, False
    cmd = [_hipcc(), *_flags_for(src), "-c", str(src), "-o", str(obj)]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")
    return obj, True


def build(jobs: int = 8, force: bool = False, verbose: bool = True) -> Path:
    """Compile every native source for gfx950 and link ``_tmx_native.so``; returns the library path."""
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    flags, headers = _common_flags(), _headers_digest()
    digests = {s.name: source_digest(s, [*flags, *_EXTRA_FLAGS.get(s.name, [])], headers) for s in srcs}
    manifest = _load_manifest()
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        results = list(ex.map(lambda s: _compile(s, digests[s.name], manifest, force), srcs))
    objs = [o for o, _ in results]
    rebuilt = sum(1 for _, r in results if r)
    manifest.update(digests)
    MANIFEST.write_text(json.dumps(manifest, indent=1, sort_keys=True))
    tree = tree_digest()
    stamp_ok = STAMP.exists() and STAMP.read_text().strip() == tree
    if not force and rebuilt == 0 and LIB_PATH.exists() and stamp_ok:
        if verbose:
            print(f"[tmx build] up to date (sources sha256 {tree[:16]}): {LIB_PATH}")
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
        "-ltorch_python",
        f"-Wl,-rpath,{lib}",
        "-o",
        str(tmp),
    ]
    proc = subprocess.run(cmd, capture_output=True, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{proc.stdout}\n{proc.stderr}")
    os.replace(tmp, LIB_PATH)
    STAMP.write_text(tree + "\n")
    if verbose:
        print(f"[tmx build] built {LIB_PATH} from {len(srcs)} sources ({rebuilt} recompiled, sha256 {tree[:16]})")
    return LIB_PATH


def main(argv: List[str] = sys.argv[1:]) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    build(jobs=args.jobs, force=args.force)


if __name__ == "__main__":
    main()
