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
# -Rpass-analysis=kernel-resource-usage: each TU's per-kernel VGPR / scratch / occupancy report
# is kept next to its object (build/<tu>.res.txt) and checked by tests/test_build_resources.py
# (round 5: a 76-B scratch object had sat unnoticed in every NTT pass)
RES_FLAG = "-Rpass-analysis=kernel-resource-usage"
CFLAGS = ["-std=c++17", "-O3", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-function",
          f"-I{ROOT / 'include'}", RES_FLAG]


def _headers():
    return list(CSRC.glob("*.hpp")) + list((ROOT / "include").glob("*.h"))


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: Path, obj: Path, cflags) -> str:
    cmd = [HIPCC, *cflags, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    if RES_FLAG in cflags:  # the device-side resource remarks only
        keep = ("Function Name", "VGPRs", "AGPRs", "ScratchSize", "Occupancy", "LDS Size")
        lines = [ln for ln in r.stderr.splitlines() if "remark:" in ln and any(k in ln for k in keep)]
        obj.with_suffix(".res.txt").write_text("\n".join(lines) + "\n")
    return src.name


def build(verbose: bool = True, jobs: int | None = None, variant: str = "",
          extra: tuple = (), only: tuple = ()) -> Path:
    """variant / extra: an experimental build (extra hipcc flags, e.g. -DPLK_NTT_MINW=4)
    into build-<variant>/ and libplk-<variant>.so, loaded with PLK_LIB=<path>. only: the
    TU stems that take the extra flags (e.g. ("msm_acc",)); the variant links the default
    build's objects for every other TU, so a one-kernel A/B compiles one file.

    Objects are rebuilt when a source or header is newer OR when the flags they were built
    with differ (a stamp file per build directory): an mtime check alone let a variant
    directory keep objects compiled with other flags or older sources (round-4 verdict,
    the libplk-g2 abort)."""
    build_dir, lib, cflags = BUILD, LIB, list(CFLAGS)
    if variant:
        build_dir, lib = PKG / f"build-{variant}", PKG / f"libplk-{variant}.so"
        cflags = cflags + list(extra)
        if only:
            build(verbose=verbose, jobs=jobs)  # the default objects the variant links
    build_dir.mkdir(exist_ok=True)
    stamp = build_dir / "flags.txt"
    flags_txt = " ".join(cflags) + "\n" + " ".join(only) + "\n"
    rebuild_all = not stamp.exists() or stamp.read_text() != flags_txt
    hdrs = _headers()
    srcs = sorted(CSRC.glob("*.hip"))
    todo = []
    objs = []
    for s in srcs:
        if variant and only and s.stem not in only:
            objs.append(BUILD / (s.stem + ".o"))
            continue
        o = build_dir / (s.stem + ".o")
        objs.append(o)
        if rebuild_all or _stale(o, [s, *hdrs]):
            todo.append((s, o))
    if todo:
        jobs = jobs or min(len(todo), max(1, (os.cpu_count() or 4)), 8)
        if verbose:
            print(f"[plk] compiling {len(todo)} HIP TU(s) for {ARCH} with {jobs} jobs", flush=True)
        if stamp.exists():
            stamp.unlink()
        with cf.ThreadPoolExecutor(jobs) as ex:
            for name in ex.map(lambda so: _compile(*so, cflags), todo):
                if verbose:
                    print(f"[plk]   {name}", flush=True)
        stamp.write_text(flags_txt)
    if todo or _stale(lib, objs):
        tmp = lib.with_suffix(".so.tmp")
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, lib)
        if verbose:
            print(f"[plk] linked {lib}", flush=True)
    return lib


if __name__ == "__main__":
    if len(sys.argv) > 1:  # build_ext.py <variant>[:tu1,tu2] <extra hipcc flags...>
        name, _, tus = sys.argv[1].partition(":")
        build(variant=name, extra=tuple(sys.argv[2:]), only=tuple(t for t in tus.split(",") if t))
    else:
        build()
    sys.exit(0)
