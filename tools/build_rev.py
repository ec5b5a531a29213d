"""Build libhuffman_amd.so from the sources of a git revision into huffman_amd/<dir>/ (an A/B baseline,
loaded with HZ_LIB_VARIANT=<dir>). Development tool; the product build is huffman_amd/build.py.
usage: python tools/build_rev.py REV DIR [-DFLAG ...]"""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huffman_amd import build as b  # noqa: E402

rev, name, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
out_dir = os.path.join(b.PKG, name)
os.makedirs(out_dir, exist_ok=True)
with tempfile.TemporaryDirectory() as td:
    src = os.path.join(td, "csrc")
    inc = os.path.join(td, "include")
    os.makedirs(src)
    os.makedirs(inc)
    for f in b.LIB_SOURCES + ["hz_internal.h"]:
        with open(os.path.join(src, f), "wb") as fh:
            fh.write(subprocess.run(["git", "show", f"{rev}:huffman_amd/csrc/{f}"], check=True, capture_output=True,
                                    cwd=b.ROOT).stdout)
    with open(os.path.join(inc, "huffman_amd.h"), "wb") as fh:
        fh.write(subprocess.run(["git", "show", f"{rev}:include/huffman_amd.h"], check=True, capture_output=True,
                                cwd=b.ROOT).stdout)
    cflags = [f for f in b.CFLAGS if not f.startswith("-I")] + [f"-I{inc}", f"-I{src}"]
    objs = []
    for f in b.LIB_SOURCES:
        o = os.path.join(td, f + ".o")
        lang = ["-x", "hip"] if f.endswith(".hip") else []
        subprocess.run([b.HIPCC] + cflags + flags + lang + ["-c", os.path.join(src, f), "-o", o], check=True,
                       capture_output=True)
        objs.append(o)
    subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(out_dir, "libhuffman_amd.so")] + objs, check=True)
print(out_dir)
