"""Build an A/B variant of the native library: one source recompiled with extra ``-D`` flags, linked with the
in-tree objects of every other source (``build/native``), into ``build/ab/<name>/_tmx_native.so``.  Load it on the GPU
box with ``TMX_NATIVE_LIB=$PWD/build/ab/<name>/_tmx_native.so`` (torchmetrics_forked_amd/ops/__init__.py).

    python tools/ab_build.py <name> <source.hip> -DFLAG=VALUE [...]
"""
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from torchmetrics_forked_amd.ops import build as B  # noqa: E402


def main() -> None:
    name, src, defs = sys.argv[1], Path(sys.argv[2]), sys.argv[3:]
    B.build(verbose=False)  # the in-tree objects are current
    out = B.BUILD_DIR.parent / "ab" / name
    out.mkdir(parents=True, exist_ok=True)
    obj = out / (src.name + ".o")
    subprocess.run([B._hipcc(), *B._common_flags(), *defs, "-c", str(src), "-o", str(obj)], check=True)
    objs = [obj if o.name == obj.name else o for o in sorted(B.BUILD_DIR.glob("*.o"))]
    _, _, lib = B._torch_paths()
    subprocess.run([B._hipcc(), "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *map(str, objs), f"-L{lib}", "-lc10", "-lc10_hip",
                    "-ltorch", "-ltorch_cpu", "-ltorch_hip", f"-Wl,-rpath,{lib}", "-o", str(out / "_tmx_native.so")], check=True)
    print(out / "_tmx_native.so")


if __name__ == "__main__":
    main()
