"""Build the gfx950 library and CLIs in-tree with hipcc (no JIT, no cache).

Outputs (git-ignored, shipped to the GPU box with the tree):
  huffman_amd/lib/libhuffman_amd.so   C ABI of include/huffman_amd.h
  huffman_amd/bin/archive             drop-in for the reference `archive`
  huffman_amd/bin/extract             drop-in for the reference `extract`
"""
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OBJ = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "lib", "libhuffman_amd.so")
BUILD_ID = os.path.join(PKG, "lib", "BUILD_ID")  # hash of the sources the library was built from
BIN = os.path.join(PKG, "bin")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

LIB_SOURCES = ["hz_kernels.hip", "hz_codebook_gpu.hip", "hz_codebook.cpp", "hz_host.cpp"]
HEADERS = [os.path.join(CSRC, "hz_internal.h"), os.path.join(INCLUDE, "huffman_amd.h")]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result", f"--offload-arch={ARCH}",
          f"-I{INCLUDE}", f"-I{CSRC}"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd[:3])} ...")
    elif verbose and (r.stdout or r.stderr):
        sys.stderr.write(r.stdout + r.stderr)


def source_id():
    """sha256 (16 hex digits) of every source and header the library is built from."""
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, f) for f in LIB_SOURCES] + HEADERS:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_variant(name, defines, verbose=False):
    """An A/B build of the library with extra -D flags into huffman_amd/lib_<name>/
    (loaded with HZ_LIB_VARIANT=lib_<name>; tools/ab.sh)."""
    obj_dir = os.path.join(PKG, "_build_" + name)
    lib = os.path.join(PKG, "lib_" + name, "libhuffman_amd.so")
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    objs = []
    for src in LIB_SOURCES:
        obj = os.path.join(obj_dir, src + ".o")
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        _run([HIPCC] + CFLAGS + defines + lang + ["-c", os.path.join(CSRC, src), "-o", obj], verbose)
        objs.append(obj)
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs, verbose)
    return lib


def build(verbose=False, force=False):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    os.makedirs(BIN, exist_ok=True)
    objs = []
    for src in LIB_SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(OBJ, src + ".o")
        objs.append(obj)
        if force or _stale(obj, [path] + HEADERS):
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            _run([HIPCC] + CFLAGS + lang + ["-c", path, "-o", obj], verbose)
    if force or _stale(LIB, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs, verbose)
    sid = source_id()
    if not os.path.exists(BUILD_ID) or open(BUILD_ID).read().strip() != sid:
        with open(BUILD_ID, "w") as f:
            f.write(sid + "\n")
    for name in ("archive", "extract"):
        src = os.path.join(CSRC, f"cli_{name}.cpp")
        out = os.path.join(BIN, name)
        if force or _stale(out, [src, LIB] + HEADERS):
            _run([HIPCC] + CFLAGS + [src, "-o", out, f"-L{os.path.dirname(LIB)}", "-lhuffman_amd",
                                     "-Wl,-rpath,$ORIGIN/../lib"], verbose)
    return LIB


if __name__ == "__main__":
    if "--variant" in sys.argv:  # python huffman_amd/build.py --variant NAME -DFLAG ...
        i = sys.argv.index("--variant")
        print(build_variant(sys.argv[i + 1], [a for a in sys.argv[i + 2:] if a.startswith("-D")], "-v" in sys.argv))
    else:
        build(verbose="-v" in sys.argv, force="-f" in sys.argv)
        print(LIB)
