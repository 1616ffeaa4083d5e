"""Build libgpmdm_hip.so in-tree (hipcc, gfx950 only).

    python -m gpmdm_amd.build          # or __graft_entry__.build()

Each translation unit is compiled with ``hipcc --offload-arch=gfx950 -O3`` and linked
into ``gpmdm_amd/libgpmdm_hip.so``; objects go to ``gpmdm_amd/_build/``.  Rebuilds only
what changed (source or header newer than the object).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "_build"
LIB = PKG / "libgpmdm_hip.so"
SOURCES = ["gp_tile.hip", "gp_tile_d1.hip", "gp_tile_d2.hip", "gp_tile_d3.hip", "gp_tile_d4.hip",
           "gp_tile_d5.hip", "pf_kernels.hip", "capi_model.hip", "capi_pf.hip", "capi_frame.hip",
           "capi_exchange.hip", "capi_replay.hip", "precompute.hip", "shard_order.hip", "torch_rng.cpp",
           "obs_cutoff.hip", "obs_cutoff_d9.hip", "memory.hip", "cutoff_image.hip"]
HEADERS = [CSRC / "common.h", CSRC / "geometry.h", CSRC / "host_image.h", CSRC / "gp_tile.h", CSRC / "pf_kernels.h",
           CSRC / "status.h", CSRC / "capi_internal.h", CSRC / "obs_cutoff.h", ROOT / "include" / "gpmdm_hip.h"]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build libgpmdm_hip.so)")


def _flags():
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-unused-function", "-munsafe-fp-atomics", f"-I{ROOT / 'include'}"]


C_HOST_SRC = ROOT / "examples" / "c_host" / "pf_main.c"
C_HOST = ROOT / "examples" / "c_host" / "pf_main"


def build_c_host(force: bool = False, verbose: bool = False) -> Path:
    """The native C host of the C ABI (examples/c_host/pf_main.c): plain gcc against
    include/gpmdm_hip.h, linked to the in-tree library by a relative rpath."""
    if not C_HOST_SRC.exists():
        return C_HOST
    deps = max(C_HOST_SRC.stat().st_mtime, (ROOT / "include" / "gpmdm_hip.h").stat().st_mtime)
    if not force and C_HOST.exists() and C_HOST.stat().st_mtime >= deps:
        return C_HOST
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", f"-I{ROOT / 'include'}", str(C_HOST_SRC),
           "-o", str(C_HOST), f"-L{PKG}", "-lgpmdm_hip", "-Wl,-rpath,$ORIGIN/../../gpmdm_amd"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return C_HOST


REPLAY_SRC = CSRC / "replay_draws.cpp"
REPLAY_LIB = PKG / "libgpmdm_replay.so"


def build_replay(force: bool = False, verbose: bool = False) -> Path:
    """The replay draws' chunk runner (csrc/replay_draws.cpp): host C++ against libtorch_cpu
    (torch's own CPU samplers), g++ with torch's headers and C++ ABI, rpath to torch/lib."""
    import torch
    tdir = Path(torch.__file__).resolve().parent
    if not force and REPLAY_LIB.exists() and REPLAY_LIB.stat().st_mtime >= max(REPLAY_SRC.stat().st_mtime,
                                                                            Path(__file__).stat().st_mtime):
        return REPLAY_LIB
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    tmp = REPLAY_LIB.with_suffix(".so.tmp")
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-pthread", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           f"-I{tdir / 'include'}", f"-I{tdir / 'include' / 'torch' / 'csrc' / 'api' / 'include'}",
           str(REPLAY_SRC), "-o", str(tmp), f"-L{tdir / 'lib'}", "-ltorch_cpu", "-lc10",
           f"-Wl,-rpath,{tdir / 'lib'}"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, REPLAY_LIB)
    return REPLAY_LIB


def build(force: bool = False, verbose: bool = False) -> Path:
    lib = _build_lib(force, verbose)
    build_c_host(force, verbose)
    build_replay(force, verbose)
    return lib


def _deps(path: Path, seen=None) -> set:
    """The file and every local header it includes (#include "..."), transitively."""
    seen = set() if seen is None else seen
    if path in seen or not path.exists():
        return seen
    seen.add(path)
    for line in path.read_text(errors="replace").splitlines():
        s = line.strip()
        if s.startswith("#include \""):
            _deps((path.parent / s.split('"')[1]).resolve(), seen)
    return seen


def _build_lib(force: bool = False, verbose: bool = False) -> Path:
    newest_hdr = max(h.stat().st_mtime for h in HEADERS)
    newest_src = max((CSRC / src).stat().st_mtime for src in SOURCES)
    if not force and LIB.exists() and LIB.stat().st_mtime >= max(newest_hdr, newest_src):
        return LIB                      # current (objects need not be present, e.g. on a GPU box)
    OBJ.mkdir(exist_ok=True)
    cc = hipcc()
    jobs = []
    for src in SOURCES:
        s = CSRC / src
        o = OBJ / (src + ".o")
        newest = max(p.stat().st_mtime for p in _deps(s.resolve()))   # the source and its headers
        if force or not o.exists() or o.stat().st_mtime < newest:
            jobs.append([cc, *_flags(), "-c", str(s), "-o", str(o)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        list(ex.map(run, jobs))
    objs = [str(OBJ / (s + ".o")) for s in SOURCES]
    if force or jobs or not LIB.exists():
        # link to a temporary name, then rename: a reader (a process loading the library, a
        # snapshot of the tree) never sees a partly written file
        tmp = LIB.with_suffix(".so.tmp")
        run([cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *objs,
             "-L/opt/rocm/lib", "-lrocsolver", "-lrocblas", "-ldl", "-Wl,-rpath,/opt/rocm/lib"])
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
