"""Builds libplk.so (the C-ABI product library) in-tree for gfx950 with hipcc.

Each csrc/*.hip is compiled to build/<name>.o in parallel (they are independent; the
381-bit arithmetic makes single TUs slow to compile), then linked into
dusk-plonk_amd/libplk.so next to this file, where plonk.py loads it from. Objects are
rebuilt only when a source or any header is newer.
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
BUILD = PKG / "build"
LIB = PKG / "libplk.so"
ARCH = os.environ.get("PLK_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-std=c++17", "-O3", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-function",
          f"-I{ROOT / 'include'}"]


def _headers():
    return list(CSRC.glob("*.hpp")) + list((ROOT / "include").glob("*.h"))


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: Path, obj: Path) -> str:
    cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return src.name


def build(verbose: bool = True, jobs: int | None = None, variant: str = "",
          extra: tuple = ()) -> Path:
    """variant / extra: an experimental build (extra hipcc flags, e.g. -DPLK_ACC_WAVES=3)
    into build-<variant>/ and libplk-<variant>.so, loaded with PLK_LIB=<path>."""
    global BUILD, LIB, CFLAGS
    if variant:
        BUILD, LIB = PKG / f"build-{variant}", PKG / f"libplk-{variant}.so"
        CFLAGS = CFLAGS + list(extra)
    BUILD.mkdir(exist_ok=True)
    hdrs = _headers()
    srcs = sorted(CSRC.glob("*.hip"))
    todo = []
    objs = []
    for s in srcs:
        o = BUILD / (s.stem + ".o")
        objs.append(o)
        if _stale(o, [s, *hdrs]):
            todo.append((s, o))
    if todo:
        jobs = jobs or min(len(todo), max(1, (os.cpu_count() or 4)), 8)
        if verbose:
            print(f"[plk] compiling {len(todo)} HIP TU(s) for {ARCH} with {jobs} jobs", flush=True)
        with cf.ThreadPoolExecutor(jobs) as ex:
            for name in ex.map(lambda so: _compile(*so), todo):
                if verbose:
                    print(f"[plk]   {name}", flush=True)
    if todo or _stale(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[plk] linked {LIB}", flush=True)
    return LIB


if __name__ == "__main__":
    if len(sys.argv) > 1:  # build_ext.py <variant> <extra hipcc flags...>
        build(variant=sys.argv[1], extra=tuple(sys.argv[2:]))
    else:
        build()
    sys.exit(0)
