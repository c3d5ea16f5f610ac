"""In-tree build of the native extension ``akka_allreduce_amd._native``.

Host C++ (engine, data plane, transports, bindings) is compiled with g++;
the gfx950 kernels with ``hipcc --offload-arch=gfx950``.  The module links the
HIP runtime and RCCL shipped inside the installed torch wheel (same sonames
as ROCm's), so one process never mixes two copies of either library.
Incremental: an object is rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shlex
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
PKG = os.path.join(ROOT, "akka_allreduce_amd")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("AKKA_OFFLOAD_ARCH", "gfx950")

HOST_SOURCES = [
    "engine/host_device.cpp",
    "engine/racecheck.cpp",
    "engine/dataplane.cpp",
    "engine/engine.cpp",
    "transport/sim_p2p.cpp",
    "transport/stream_link.cpp",
    "transport/reactive_link.cpp",
    "transport/rccl_p2p.cpp",
    "transport/ipc_lane.cpp",
    "transport/ipc_p2p.cpp",
    "transport/onesided.cpp",
    "transport/link_probe.cpp",
    "kernels/hip_device.cpp",
    "runtime/watchdog.cpp",
    "bindings/bindings.cpp",
    "bindings/bind_onesided.cpp",
    "bindings/bind_probe.cpp",
]
HIP_SOURCES = ["kernels/kernels.hip", "kernels/ipc.hip", "kernels/onesided.hip", "kernels/probe.hip"]


def ext_path() -> str:
    return os.path.join(PKG, "_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_lib() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        raise RuntimeError("torch is required to locate the HIP runtime / RCCL it ships")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _headers() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def _stale(obj: str, src: str, headers: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in headers)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, sanitize: str | None = None) -> str:
    """Compile and link.  ``sanitize`` (e.g. ``"address,undefined"``) builds an
    instrumented HOST-code variant into ``build/native-<san>/`` (never the
    in-tree module); device code is not instrumented (no GPU sanitizers on
    this pool).  Load it with ``AKKA_NATIVE_PATH=<path>``."""
    import pybind11

    tag = sanitize.replace(",", "-") if sanitize else None
    bdir = os.path.join(ROOT, "build", f"native-{tag}") if tag else BUILD
    os.makedirs(bdir, exist_ok=True)
    py_inc = sysconfig.get_paths()["include"]
    opt = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={sanitize}"] if sanitize else ["-O3"]
    common = ["-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-I" + CSRC]
    host_flags = opt + common + [
        "-D__HIP_PLATFORM_AMD__",
        "-I" + os.path.join(ROCM, "include"),
        "-I" + pybind11.get_include(),
        "-I" + py_inc,
        "-fvisibility=hidden",
    ]
    hip_flags = ["-O3"] + common + [f"--offload-arch={ARCH}", "-I" + os.path.join(ROCM, "include")]
    headers = _headers()
    steps = []
    objs = []
    for rel in HOST_SOURCES:
        src = os.path.join(CSRC, rel)
        obj = os.path.join(bdir, rel.replace("/", "_") + ".o")
        objs.append(obj)
        if force or _stale(obj, src, headers):
            steps.append(["g++", *host_flags, "-c", src, "-o", obj])
    for rel in HIP_SOURCES:
        src = os.path.join(CSRC, rel)
        obj = os.path.join(bdir, rel.replace("/", "_") + ".o")
        objs.append(obj)
        if force or _stale(obj, src, headers):
            steps.append([os.path.join(ROCM, "bin", "hipcc"), *hip_flags, "-c", src, "-o", obj])
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for f in [ex.submit(_run, s, verbose) for s in steps]:
            f.result()
    out = os.path.join(bdir, "_native" + sysconfig.get_config_var("EXT_SUFFIX")) if tag else ext_path()
    if force or steps or not os.path.exists(out):
        tlib = _torch_lib()
        linker = ["g++", f"-fsanitize={sanitize}"] if sanitize else [os.path.join(ROCM, "bin", "hipcc")]
        link = [
            *linker,
            "-shared",
            "-fPIC",
            *objs,
            "-o",
            out + ".tmp",
            "-L" + tlib,
            "-lamdhip64",
            "-lrccl",
            f"-Wl,-rpath,{tlib}",
        ]
        _run(link, verbose)
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    san = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--sanitize=")), None)
    path = build(force="--force" in sys.argv, verbose="-v" in sys.argv, sanitize=san)
    print(path)
