"""Build libchoco_codec.so (HIP, gfx950) in-tree with hipcc.

The library is a plain C-ABI shared object (include/choco_codec.h): no torch
headers, no Python.  Objects are compiled in parallel and linked once; a
rebuild is skipped when the .so is newer than every source.
"""
import concurrent.futures
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libchoco_codec.so")
ARCH = os.environ.get("CHOCO_OFFLOAD_ARCH", "gfx950")

HIPCC_FLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-ffp-contract=off",          # keep the reference's fp32 rounding sequence
    "-fvisibility=hidden",        # only CHOCO_API symbols are exported
    "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
]


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X codec must be built with ROCm's hipcc")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force=False, verbose=False, jobs=None, defines=(), lib=None):
    """Build the codec.  `defines`/`lib` build a diagnostic variant (tools/) into its
    own object dir and .so; the product library is always the default LIB."""
    out = lib or LIB
    if not force and not defines and not _stale():
        return LIB
    hipcc = _hipcc()
    tag = "_".join(d.replace("=", "") for d in defines)
    objdir = os.path.join(PKG, "build_obj" + ("_" + tag if tag else ""))
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)

    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    flags_stamp = os.path.join(objdir, "flags.txt")
    flags = " ".join(HIPCC_FLAGS + [f"-D{d}" for d in defines])
    same_flags = os.path.exists(flags_stamp) and open(flags_stamp).read() == flags

    macros = [d.split("=")[0] for d in defines]
    in_headers = any(m in open(h).read() for h in headers for m in macros)

    def compile_one(src):
        # a variant's macros that only one source names: the other objects are the
        # product build's (built first, below)
        if defines and not in_headers and not any(m in open(src).read() for m in macros):
            return os.path.join(PKG, "build_obj", os.path.basename(src) + ".o")
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        # an object newer than its source and every header, built with the same flags, is kept
        if same_flags and os.path.exists(obj):
            t = os.path.getmtime(obj)
            if all(os.path.getmtime(d) <= t for d in [src] + headers):
                return obj
        cmd = [hipcc, *HIPCC_FLAGS, *[f"-D{d}" for d in defines], "-I", INCLUDE, "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-8000:]}")
        if verbose and r.stderr:
            sys.stderr.write(r.stderr)
        return obj

    srcs = sources()
    if defines:
        build_library(jobs=jobs)  # the product objects a variant reuses
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 2)), 8)
    with concurrent.futures.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    with open(flags_stamp, "w") as f:
        f.write(flags)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-8000:]}")
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
