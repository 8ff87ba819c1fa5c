"""Builds libdkgpu.so in-tree (hipcc, gfx950). Used by __graft_entry__.build() and the tests."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libdkgpu.so")
OBJ = os.path.join(HERE, "..", "build", "obj")   # kept between builds: only stale objects recompile
SOURCES = ["dk_host.cpp", "dk_expr.cpp", "dk_comm.cpp", "dk_kernels.hip", "dk_arrow.hip", "dk_dv.hip", "dk_encode.hip"]
HEADERS = ["dk_device.h", "dk_thrift.h", "dk_uri.h", "dk_expr.h"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(HERE, "..", "include", "dkgpu.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
             "-Wall", "-Wno-unused-function", "-Wno-unused-result", "-Wno-unused-value",
             "-I", os.path.join(HERE, "..", "include")]
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = max(os.path.getmtime(d) for d in [os.path.join(CSRC, f) for f in HEADERS]
                + [os.path.join(HERE, "..", "include", "dkgpu.h")])
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(OBJ, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        if not force and os.path.exists(obj) and os.path.getmtime(obj) > max(hdr_t, os.path.getmtime(os.path.join(CSRC, src))):
            continue
        cmd = [hipcc] + flags + ["-c", os.path.join(CSRC, src), "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), obj))
    bad = [p.wait() for p, _ in procs]
    if any(bad):
        raise subprocess.CalledProcessError(max(bad), "hipcc")
    for _, obj in procs:
        os.replace(obj + ".tmp", obj)
    cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
