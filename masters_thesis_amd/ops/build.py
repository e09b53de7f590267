"""In-tree build of the HIP extension ``masters_thesis_amd/_C*.so`` for gfx950.

Each ``csrc/*.hip`` kernel file is compiled by ``hipcc --offload-arch=gfx950`` to an
object (no torch headers, seconds per file); ``csrc/bindings.cpp`` is the only TU that
includes torch; everything is linked with ``hipcc -shared``.  Objects are cached under
``build/`` keyed by a hash of (source, headers, flags), so a rebuild after editing one
kernel recompiles one file.  No hipify, no CUDA paths: gfx950 only.

    python -m masters_thesis_amd.ops.build [-v] [--force] [--debug]
    python -m masters_thesis_amd.ops.build --sanitize      # host runtime under ASan+UBSan and TSan (no GPU)
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List

REPO = Path(__file__).resolve().parents[2]
CSRC = REPO / "csrc"
PKG = REPO / "masters_thesis_amd"
BUILD = REPO / "build" / "hip"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm required to build masters_thesis_amd._C)")


def _torch_flags():
    import torch
    import torch.utils.cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths()]
    inc.append(f"-I{sysconfig.get_paths()['include']}")
    libdir = str(Path(torch.__file__).parent / "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
            "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    libs = [f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            f"-Wl,-rpath,{libdir}"]
    return inc, defs, libs


def _digest(paths: List[Path], flags: List[str]) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(p.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def ext_path() -> Path:
    return PKG / f"_C{EXT_SUFFIX}"


def sources() -> List[Path]:
    return sorted(CSRC.glob("*.hip"))


def host_sources() -> List[Path]:
    """Host-only C++ runtime pieces (prefetcher, ...): plain C++17, no HIP, no torch."""
    return sorted((CSRC / "host").glob("*.cpp"))


def _compile(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)


def build(verbose: bool = False, force: bool = False, debug: bool = False, jobs: int = 0) -> Path:
    hipcc = _hipcc()
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    opt = ["-O0", "-g"] if debug else ["-O3"]
    kflags = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", *opt, "-munsafe-fp-atomics", f"-I{CSRC}"]
    inc, defs, libs = _torch_flags()
    bflags = ["-std=c++17", "-fPIC", "-O2", *inc, *defs, f"-I{CSRC}"]

    jobs_list = []
    objs = []
    for src in sources():
        key = _digest([src, *headers], kflags)
        obj = BUILD / f"{src.stem}-{key}.o"
        objs.append(obj)
        if force or not obj.exists():
            jobs_list.append(([hipcc, *kflags, "-c", str(src), "-o", str(obj)], obj))
    hflags = ["-std=c++17", "-fPIC", "-O3", "-pthread", f"-I{CSRC}"]
    cxx = shutil.which("g++") or shutil.which("c++") or hipcc
    for src in host_sources():
        key = _digest([src, *headers], hflags)
        obj = BUILD / f"host_{src.stem}-{key}.o"
        objs.append(obj)
        if force or not obj.exists():
            jobs_list.append(([cxx, *hflags, "-c", str(src), "-o", str(obj)], obj))
    bsrc = CSRC / "bindings.cpp"
    bkey = _digest([bsrc], bflags)
    bobj = BUILD / f"bindings-{bkey}.o"
    objs.append(bobj)
    if force or not bobj.exists():
        jobs_list.append(([hipcc, *bflags, "-c", str(bsrc), "-o", str(bobj)], bobj))

    out = ext_path()
    link_key = hashlib.sha256("\n".join(o.name for o in objs).encode()).hexdigest()[:16]
    stamp = BUILD / "link.stamp"
    if not jobs_list and out.exists() and stamp.exists() and stamp.read_text() == link_key and not force:
        if verbose:
            print(f"[build] up to date: {out}")
        return out

    n = jobs or min(len(jobs_list) or 1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, n)) as ex:
        futs = [ex.submit(_compile, cmd, verbose) for cmd, _ in jobs_list]
        for f in cf.as_completed(futs):
            f.result()
    tmp = out.with_name(out.name + f".tmp{os.getpid()}")
    _compile([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *[str(o) for o in objs], "-o", str(tmp), *libs, "-pthread"],
             verbose)
    os.replace(tmp, out)
    stamp.write_text(link_key)
    # drop stale objects of older source versions
    keep = {o.name for o in objs}
    for o in BUILD.glob("*.o"):
        if o.name not in keep:
            o.unlink(missing_ok=True)
    if verbose:
        print(f"[build] wrote {out}")
    return out


SANITIZERS = {"asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer"], "tsan": ["-fsanitize=thread"]}


def build_host_sanitized(kinds=("asan", "tsan"), verbose: bool = False) -> List[Path]:
    """Host-only C++ runtime (csrc/host/*.cpp) + its stress drivers (csrc/host/tests/*.cpp) under the
    sanitizers, as plain g++ executables (no HIP, no torch): race / memory-error detection for the native
    runtime pieces.  Returns the executables (build/sanitize/<driver>_<kind>)."""
    # ROCm's clang++ first: its TSan runtime intercepts libstdc++'s condition variables (gcc 11's libtsan
    # reports false 'double lock' / races on std::condition_variable waits)
    rocm_clang = Path("/opt/rocm/lib/llvm/bin/clang++")
    cxx = str(rocm_clang) if rocm_clang.exists() else (shutil.which("clang++") or shutil.which("g++"))
    if cxx is None:
        raise RuntimeError("no host C++ compiler for the sanitizer builds")
    out_dir = REPO / "build" / "sanitize"
    out_dir.mkdir(parents=True, exist_ok=True)
    outs = []
    for drv in sorted((CSRC / "host" / "tests").glob("*.cpp")):
        for kind in kinds:
            exe = out_dir / f"{drv.stem}_{kind}"
            cmd = [cxx, "-std=c++17", "-O1", "-g", *SANITIZERS[kind], "-pthread", str(drv),
                   *[str(p) for p in host_sources()], "-o", str(exe)]
            if verbose:
                print("[build]", " ".join(cmd))
            subprocess.run(cmd, check=True)
            outs.append(exe)
    return outs


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--sanitize", action="store_true", help="host runtime sanitizer builds (+ run them)")
    a = ap.parse_args(argv)
    if a.sanitize:
        for exe in build_host_sanitized(verbose=a.verbose):
            r = subprocess.run([str(exe)], capture_output=True, text=True)
            print(f"{exe.name}: rc={r.returncode} {r.stdout.strip()} {r.stderr.strip()[-2000:]}")
        return
    print(build(verbose=a.verbose, force=a.force, debug=a.debug, jobs=a.jobs))


if __name__ == "__main__":
    main()
