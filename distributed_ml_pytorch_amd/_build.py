"""In-tree build of the gfx950 HIP extension (`distributed_ml_pytorch_amd/_native*.so`).

Drives ``hipcc --offload-arch=gfx950`` directly (no hipify, no multi-arch):
each ``csrc/*.hip`` kernel file compiles to an object in parallel, the single
``bindings.cpp`` (the only TU that sees torch headers) compiles once, and they
link into one Python extension that resolves ``libamdhip64.so.7`` to the HIP
runtime torch has already loaded.

Incremental: an object is rebuilt only when its source or any header in
``csrc/`` is newer.  ``python -m distributed_ml_pytorch_amd._build`` builds.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD = PKG_DIR.parent / "build" / "native"
ARCH = os.environ.get("DMP_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_native"


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def ext_path() -> Path:
    return PKG_DIR / (EXT_NAME + _ext_suffix())


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = Path(rocm) / "bin" / "hipcc"
    if cand.exists():
        return str(cand)
    found = shutil.which("hipcc")
    if not found:
        raise RuntimeError("hipcc not found (ROCm toolchain required to build the extension)")
    return found


def _torch_flags():
    import torch
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    libdirs = [str(Path(torch.__file__).parent / "lib")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
        "-DUSE_ROCM=1",
        "-DHIPBLAS_V2",
    ]
    try:
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            defs += list(ce._get_pybind11_abi_build_flags())
    except Exception:  # pragma: no cover - torch internals moved
        pass
    return inc, libdirs, defs


def _needs(obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> Path:
    hipcc = _hipcc()
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", str(CSRC),
              "-Wno-unused-result", "-Wno-deprecated-declarations"]
    objs = []
    jobs_list = []
    for src in sorted(CSRC.glob("*.hip")):
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _needs(obj, [src, *headers]):
            jobs_list.append([hipcc, *common, "-x", "hip", "-c", str(src), "-o", str(obj)])
    inc, libdirs, defs = _torch_flags()
    py_inc = sysconfig.get_paths()["include"]
    bsrc = CSRC / "bindings.cpp"
    bobj = BUILD / "bindings.o"
    objs.append(bobj)
    if force or _needs(bobj, [bsrc, *headers]):
        cmd = ["g++", "-O2", "-fPIC", "-std=c++17", "-I", str(CSRC), "-I", py_inc,
               "-Wno-unused-result", "-Wno-deprecated-declarations", "-Wno-unknown-pragmas",
               "-Wno-ignored-attributes"]
        for i in inc:
            cmd += ["-isystem", i]
        cmd += defs + ["-D__HIP_PLATFORM_AMD__=1", "-c", str(bsrc), "-o", str(bobj)]
        jobs_list.append(cmd)
    # runtime (host-only C++) sources
    for src in sorted(CSRC.glob("*.cc")):
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or _needs(obj, [src, *headers]):
            jobs_list.append(["g++", "-O3", "-fPIC", "-std=c++17", "-pthread", "-I", str(CSRC),
                              "-c", str(src), "-o", str(obj)])
    n = jobs or min(8, max(1, os.cpu_count() or 1), max(1, len(jobs_list)))
    if jobs_list:
        with cf.ThreadPoolExecutor(n) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))
    out = ext_path()
    if force or jobs_list or not out.exists():
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(out),
                *map(str, objs)]
        for d in libdirs:
            link += ["-L", d, f"-Wl,-rpath,{d}"]
        link += ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
                 "-lamdhip64", "-pthread"]
        _run(link, verbose)
    return out


if __name__ == "__main__":
    p = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    print(p)
