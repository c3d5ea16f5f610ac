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


def source_hash(root: str | None = None) -> str | None:
    """sha256 over every source and header the module is built from (names +
    contents) and the target arch, or None when the sources are not there
    (an installed copy without ``csrc/``).  Contents, not mtimes: a snapshot
    copied to another machine keeps its hash whatever its timestamps."""
    import hashlib

    csrc = os.path.join(root or ROOT, "csrc")
    files = [os.path.join(csrc, r) for r in HOST_SOURCES + HIP_SOURCES]
    files += sorted(glob.glob(os.path.join(csrc, "**", "*.h"), recursive=True))
    if not all(os.path.exists(f) for f in files[: len(HOST_SOURCES) + len(HIP_SOURCES)]):
        return None
    h = hashlib.sha256(ARCH.encode())
    for f in files:
        if not os.path.exists(f):
            continue
        h.update(os.path.relpath(f, csrc).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def hash_path(ext: str | None = None) -> str:
    """Sidecar file holding the source hash the module at ``ext`` was linked from."""
    return (ext or ext_path()) + ".srchash"


def stale_reason(ext: str | None = None, root: str | None = None) -> str | None:
    """Why the module at ``ext`` does not match the sources (None: it does,
    or there are no sources to compare with)."""
    ext = ext or ext_path()
    if not os.path.exists(ext):
        return "not built"
    want = source_hash(root)
    if want is None:
        return None
    try:
        with open(hash_path(ext)) as f:
            have = f.read().strip()
    except OSError:
        return "no source hash recorded next to the module"
    return None if have == want else "sources changed since the module was built"


def have_compiler() -> bool:
    import shutil

    return os.path.exists(os.path.join(ROCM, "bin", "hipcc")) and shutil.which("g++") is not None


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
    this pool).  Load it with ``AKKA_NATIVE_PATH=<path>``.

    Objects are rebuilt when their source or a header is newer; a module
    whose recorded source hash (``hash_path``) disagrees with the sources
    while no timestamp says so (a copied tree) is rebuilt from scratch.
    Concurrent builds (several ranks importing at once) serialise on a lock
    file and the later ones find the module current."""
    import fcntl

    tag = sanitize.replace(",", "-") if sanitize else None
    bdir = os.path.join(ROOT, "build", f"native-{tag}") if tag else BUILD
    os.makedirs(bdir, exist_ok=True)
    with open(os.path.join(bdir, ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            return _build_locked(bdir, tag, force, jobs, verbose, sanitize)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(bdir: str, tag, force: bool, jobs, verbose: bool, sanitize) -> str:
    import pybind11

    out = os.path.join(bdir, "_native" + sysconfig.get_config_var("EXT_SUFFIX")) if tag else ext_path()
    digest = source_hash()
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

    def plan(everything: bool):
        steps, objs = [], []
        for rel in HOST_SOURCES + HIP_SOURCES:
            src = os.path.join(CSRC, rel)
            obj = os.path.join(bdir, rel.replace("/", "_") + ".o")
            objs.append(obj)
            if everything or _stale(obj, src, headers):
                cc = [os.path.join(ROCM, "bin", "hipcc"), *hip_flags] if rel.endswith(".hip") else ["g++", *host_flags]
                steps.append([*cc, "-c", src, "-o", obj])
        return steps, objs

    steps, objs = plan(force)
    mismatch = os.path.exists(out) and stale_reason(out) is not None
    if mismatch and not steps:
        steps, objs = plan(True)  # the hash says the module is old, no timestamp says which object
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for f in [ex.submit(_run, s, verbose) for s in steps]:
            f.result()
    if force or steps or not os.path.exists(out) or mismatch:
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
        if digest is not None:
            # written after the module: a crash in between leaves a mismatch
            # (rebuild), never a new hash next to an old module
            with open(hash_path(out) + ".tmp", "w") as f:
                f.write(digest + "\n")
            os.replace(hash_path(out) + ".tmp", hash_path(out))
    return out


if __name__ == "__main__":
    san = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--sanitize=")), None)
    path = build(force="--force" in sys.argv, verbose="-v" in sys.argv, sanitize=san)
    print(path)
