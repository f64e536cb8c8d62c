"""Build librecsys_hip.so in-tree: every csrc/*.hip compiled for gfx950 with hipcc, then linked.

The library is plain C-ABI (include/recsys_hip.h); Python reaches it through ctypes
(recommender_amd/_lib.py). No torch headers are involved, so the build is a few hipcc calls.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OUT_DIR = PKG / "_lib"
LIB = OUT_DIR / "librecsys_hip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RS_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: no silent a*b+c → fma contraction, so the optimizer updates round exactly
# like the fp32 oracle (explicit fmaf / MFMA are used where fused arithmetic is wanted).
CFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off",
    "-munsafe-fp-atomics", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
    "-Wno-unused-lambda-capture", f"-I{ROOT / 'include'}",
]


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _obj(src: Path) -> Path:
    return OUT_DIR / "obj" / (src.stem + ".o")


def _needs_build(src: Path, obj: Path) -> bool:
    if not obj.exists():
        return True
    deps = [src, *CSRC.glob("*.hpp"), ROOT / "include" / "recsys_hip.h", Path(__file__)]
    return any(d.stat().st_mtime > obj.stat().st_mtime for d in deps)


def _compile(src: Path) -> Path:
    obj = _obj(src)
    obj.parent.mkdir(parents=True, exist_ok=True)
    cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> Path:
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    todo = [s for s in srcs if force or _needs_build(s, _obj(s))]
    if todo:
        jobs = min(len(todo), int(os.environ.get("MAX_JOBS", "8")), 16)
        with cf.ThreadPoolExecutor(jobs) as ex:
            for obj in ex.map(_compile, todo):
                if verbose:
                    print(f"[build] compiled {obj.name}", file=sys.stderr)
    objs = [_obj(s) for s in srcs]
    if force or todo or not LIB.exists() or any(o.stat().st_mtime > LIB.stat().st_mtime for o in objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[build] linked {LIB}", file=sys.stderr)
    return LIB


def build_variant(name: str, flags: list[str]) -> Path:
    """A/B helper: the whole library rebuilt with extra -D flags into _lib/variants/<name>.so
    (loaded by setting RS_LIB=<path>; the product path always loads librecsys_hip.so)."""
    vdir = OUT_DIR / "variants" / name
    vdir.mkdir(parents=True, exist_ok=True)

    def one(src: Path) -> Path:
        obj = vdir / (src.stem + ".o")
        cmd = [HIPCC, *CFLAGS, *flags, "-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
        return obj

    with cf.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, _sources()))
    out = OUT_DIR / "variants" / f"{name}.so"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(out), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":
        print(build_variant(sys.argv[2], sys.argv[3:]))
    else:
        build(force="--force" in sys.argv)
