"""In-tree build of the native libraries (no hipify, no JIT cache).

Two shared objects are produced next to this file, in ``ops/_lib/``:

``libmda_hip.so``
    Every ``csrc/*.hip`` translation unit compiled by ``hipcc
    --offload-arch=gfx950`` (CDNA4 device code + host launchers with a plain C
    ABI) and linked with ``hipcc -shared``.
``libmda_host.so``
    The CPU-side runtime (``csrc/host/*.cpp``): CRD negative sampler, batch
    gather for the device-resident data loader.  Built with ``g++``.

Both are loaded with :mod:`ctypes` (see ``_ext.py``).  A content hash of the
sources + flags is stored beside each library; a stale or missing library is
rebuilt on first use, so a fresh GPU box (same image, hipcc present) never runs
without native code.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
ARCH = os.environ.get("MDA_OFFLOAD_ARCH", "gfx950")

HIP_LIB = os.path.join(LIBDIR, "libmda_hip.so")
HOST_LIB = os.path.join(LIBDIR, "libmda_host.so")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
    "-munsafe-fp-atomics", "-ffp-contract=fast",
    "-Wno-unused-result", "-Wno-unused-parameter",
    f"-I{CSRC}",
]
HOST_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-march=x86-64-v2", "-fopenmp", f"-I{CSRC}"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP kernels)")


def _sources(kind: str):
    if kind == "hip":
        d, ext = CSRC, ".hip"
    else:
        d, ext = os.path.join(CSRC, "host"), ".cpp"
    if not os.path.isdir(d):
        return []
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(ext))


def _headers():
    out = []
    for root, _, files in os.walk(CSRC):
        out += [os.path.join(root, f) for f in files if f.endswith((".h", ".hpp", ".cuh", ".inc"))]
    return sorted(out)


def _digest(kind: str) -> str:
    h = hashlib.sha256()
    flags = HIPCC_FLAGS if kind == "hip" else HOST_FLAGS
    h.update(" ".join(flags).encode())
    for p in _sources(kind) + _headers():
        h.update(p.replace(CSRC, "").encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stamp(lib: str) -> str:
    return lib + ".sha256"


def is_fresh(kind: str) -> bool:
    lib = HIP_LIB if kind == "hip" else HOST_LIB
    if not os.path.exists(lib) or not os.path.exists(_stamp(lib)):
        return False
    with open(_stamp(lib)) as f:
        return f.read().strip() == _digest(kind)


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build command failed:\n  {}\n{}".format(" ".join(cmd), r.stdout[-8000:]))
    return r.stdout


def build(kind: str = "all", verbose: bool = False, jobs: int | None = None) -> list:
    """Build the requested libraries if stale.  Returns the list of libraries built."""
    os.makedirs(LIBDIR, exist_ok=True)
    built = []
    kinds = ["hip", "host"] if kind == "all" else [kind]
    jobs = jobs or max(1, min(8, (os.cpu_count() or 4)))
    for k in kinds:
        if is_fresh(k):
            continue
        lib = HIP_LIB if k == "hip" else HOST_LIB
        srcs = _sources(k)
        if not srcs:
            continue
        objdir = os.path.join(LIBDIR, f"obj_{k}")
        os.makedirs(objdir, exist_ok=True)
        if k == "hip":
            cc, flags = _hipcc(), HIPCC_FLAGS
        else:
            cc, flags = (shutil.which("g++") or "g++"), HOST_FLAGS

        def compile_one(src):
            obj = os.path.join(objdir, os.path.basename(src) + ".o")
            cmd = [cc] + flags + ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            _run(cmd)
            return obj

        with ThreadPoolExecutor(max_workers=jobs) as ex:
            objs = list(ex.map(compile_one, srcs))
        tmp = lib + f".tmp{os.getpid()}"
        if k == "hip":
            link = [cc, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", tmp] + objs
        else:
            link = [cc, "-shared", "-fPIC", "-fopenmp", "-o", tmp] + objs
        _run(link)
        os.replace(tmp, lib)
        with open(_stamp(lib), "w") as f:
            f.write(_digest(k))
        built.append(lib)
        if verbose:
            print(f"built {lib}", flush=True)
    return built


SAN_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17", "-fopenmp",
             "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", f"-I{CSRC}"]


def build_host_sanitized(out_dir: str | None = None) -> str:
    """Build ``csrc/host/*.cpp`` + ``csrc/host/selftest/host_selftest.cpp``
    into ONE executable under AddressSanitizer + UBSan.  CPU only:
    GPU sanitizers are not available on the MI355X pool.  Returns its path;
    running it exits 0 when every invariant held and no sanitizer fired."""
    out_dir = out_dir or os.path.join(LIBDIR, "san")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "host_selftest_asan")
    srcs = _sources("host") + [os.path.join(CSRC, "host", "selftest", "host_selftest.cpp")]
    cc = shutil.which("g++") or "g++"
    _run([cc] + SAN_FLAGS + srcs + ["-o", exe])
    return exe


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "asan":
        exe = build_host_sanitized()
        r = subprocess.run([exe])
        sys.exit(r.returncode)
    out = build(sys.argv[1] if len(sys.argv) > 1 else "all", verbose=True)
    print("up to date" if not out else "\n".join(out))
