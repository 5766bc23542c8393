"""Native build driver: compiles every HIP kernel for gfx950 and the C++ runtime pieces.

Two in-tree shared objects are produced (they travel to GPU boxes with the repo snapshot):

* ``ome_amd/_lib/libome_kernels.so`` — all ``csrc/kernels/*.hip`` device code with a C ABI
  (``ome_*`` launchers that take raw pointers + a ``hipStream_t``), bound from Python by
  ``ome_amd.ops._native`` through ctypes.  No torch headers are involved, so a full rebuild
  takes seconds and the launchers are graph-capture safe (they only enqueue on the stream).
* ``ome_amd/_lib/libomeio.so`` — the C++ artifact I/O + runtime helpers (``csrc/omeio``):
  safetensors header parser, multi-threaded pread -> pinned-host -> HBM loader,
  paged-KV block allocator, radix prefix cache.
* ``ome_amd/_lib/libome_comm.so`` — xGMI peer-to-peer collectives (``csrc/comm``).

Usage: ``python -m ome_amd.build [--force] [--jobs N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "_lib"
OBJDIR = ROOT / "build" / "obj"
ARCH = os.environ.get("OME_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build ome_amd kernels)")


HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-unused-function"]


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(cmd: list[str]) -> tuple[list[str], int, str]:
    p = subprocess.run(cmd, capture_output=True, text=True)
    return cmd, p.returncode, p.stdout + p.stderr


def _build_lib(name: str, sources: list[Path], headers: list[Path], compiler: str, flags: list[str],
               link_flags: list[str], force: bool, jobs: int) -> Path:
    OBJDIR.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    objs, cmds = [], []
    for src in sources:
        obj = OBJDIR / f"{name}_{src.stem}.o"
        objs.append(obj)
        if force or _stale(obj, [src, *headers]):
            cmds.append([compiler, *flags, f"-I{src.parent}", f"-I{CSRC}", "-c", str(src), "-o", str(obj)])
    if cmds:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for cmd, rc, out in ex.map(_compile, cmds):
                if rc != 0:
                    raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{out}")
    lib = LIBDIR / f"lib{name}.so"
    if force or cmds or _stale(lib, objs):
        cmd = [compiler, "-shared", "-fPIC", *[str(o) for o in objs], "-o", str(lib), *link_flags]
        if "hipcc" in compiler:
            cmd.insert(3, f"--offload-arch={ARCH}")
        _, rc, out = _compile(cmd)
        if rc != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{out}")
    _check_loadable(lib)
    return lib


def _check_loadable(lib: Path) -> None:
    """dlopen the fresh library with every symbol resolved: a kernel template whose host stub was
    silently dropped links fine but fails here (and would fail on the GPU box)."""
    import ctypes

    try:
        ctypes.CDLL(str(lib), mode=os.RTLD_NOW | os.RTLD_LOCAL)
    except OSError as e:
        raise RuntimeError(f"{lib.name} does not load: {e}") from e


def build(force: bool = False, jobs: int | None = None, verbose: bool = True,
          only: tuple[str, ...] | None = None) -> list[Path]:
    """Build the native libraries (``only``: a subset of ome_kernels / omeio / ome_comm)."""
    jobs = jobs or min(8, os.cpu_count() or 4)
    hipcc = _hipcc()
    built = []
    kdir = CSRC / "kernels"
    want = set(only or ("ome_kernels", "omeio", "ome_comm"))
    if "ome_kernels" in want:
        built.append(_build_lib("ome_kernels", sorted(kdir.glob("*.hip")), sorted(kdir.glob("*.h")), hipcc,
                                HIP_FLAGS, [], force, jobs))
    iodir = CSRC / "omeio"
    io_src = sorted(iodir.glob("*.cpp"))
    if io_src and "omeio" in want:
        built.append(_build_lib("omeio", io_src, sorted(iodir.glob("*.h")), hipcc,
                                [f for f in HIP_FLAGS if not f.startswith("--offload")] + ["-pthread", "-D__HIP_PLATFORM_AMD__"],
                                ["-pthread", "-L/opt/rocm/lib", "-lamdhip64", "-lcrypto"], force, jobs))
    cdir = CSRC / "comm"
    comm_src = sorted(cdir.glob("*.hip"))
    if comm_src and "ome_comm" in want:
        built.append(_build_lib("ome_comm", comm_src, sorted(cdir.glob("*.h")) + [kdir / "common.h"], hipcc,
                                HIP_FLAGS + [f"-I{kdir}"], [], force, jobs))
    if verbose:
        for b in built:
            print(f"[ome_amd.build] {b.relative_to(ROOT)}  ({b.stat().st_size // 1024} KiB)")
    return built


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
