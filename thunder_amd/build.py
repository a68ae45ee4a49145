"""Builds thunder_amd/libthunder_amd.so from csrc/*.hip with hipcc for gfx950.

In-tree build (the .so travels to the GPU box with the repo snapshot).  Object
files are cached under build/ and rebuilt when a source or header is newer.
"""
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(HERE, "libthunder_amd.so")
ARCH = os.environ.get("THX_OFFLOAD_ARCH", "gfx950")
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
            "-Wno-unused-function", "-munsafe-fp-atomics"]


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build the gfx950 kernels")


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))


def build(verbose=False, jobs=8):
    hipcc = _hipcc()
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdr_mtime = max(os.path.getmtime(h) for h in _headers())
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_mtime):
            todo.append((s, o))

    def _compile(so):
        s, o = so
        cmd = [hipcc, *CXXFLAGS, "-c", s, "-o", o]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {s}:\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr)
        return o

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_compile, todo))
    if todo or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        tmp = LIB + ".tmp"
        r = subprocess.run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs,
                            "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lrccl", "-lhipfft", "-o", tmp],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
