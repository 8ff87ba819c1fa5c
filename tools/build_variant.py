"""Build a variant of libdkgpu.so from delta_amd/csrc with some sources replaced (A/B of kernel
changes in one GPU call: load it with DK_LIB_PATH=<out>).
Usage: python tools/build_variant.py OUT.so [overlay_dir]   (overlay files replace csrc files)"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "delta_amd", "csrc")


def main():
    out = os.path.abspath(sys.argv[1])
    overlay = sys.argv[2] if len(sys.argv) > 2 else None
    base = tempfile.mkdtemp(prefix="dkv_")
    d = os.path.join(base, "delta_amd", "csrc")          # keeps "../../include/dkgpu.h" resolvable
    os.makedirs(d)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(base, "include"))
    try:
        for f in os.listdir(CSRC):
            if f.endswith((".h", ".hip", ".cpp")):
                shutil.copy(os.path.join(CSRC, f), d)
        if overlay:
            for f in os.listdir(overlay):
                if f.endswith((".h", ".hip", ".cpp")):
                    shutil.copy(os.path.join(overlay, f), d)
        flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-w", "-I", os.path.join(ROOT, "include")]
        flags += os.environ.get("DK_VARIANT_FLAGS", "").split()
        procs, objs = [], []
        sys.path.insert(0, ROOT)
        from delta_amd.build import SOURCES
        for src in SOURCES:
            obj = os.path.join(d, src + ".o")
            procs.append(subprocess.Popen(["/opt/rocm/bin/hipcc"] + flags + ["-c", os.path.join(d, src), "-o", obj]))
            objs.append(obj)
        if any(p.wait() for p in procs):
            raise SystemExit("compile failed")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
    finally:
        shutil.rmtree(base, ignore_errors=True)


if __name__ == "__main__":
    main()
