"""Build an A/B variant of libhuffman_amd.so with extra -D flags into huffman_amd/<dir>/ (load it with
HZ_LIB_VARIANT=<dir>). Development tool: the product build is huffman_amd/build.py.
usage: python tools/build_variant.py DIR -DNAME=VALUE ..."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huffman_amd import build as b  # noqa: E402

out_dir = os.path.join(b.PKG, sys.argv[1])
flags = sys.argv[2:]
os.makedirs(out_dir, exist_ok=True)
objs = []
for src in b.LIB_SOURCES:
    o = os.path.join("/tmp", f"hzvar_{sys.argv[1]}_{src}.o")
    objs.append(o)
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    subprocess.run([b.HIPCC] + b.CFLAGS + flags + lang + ["-c", os.path.join(b.CSRC, src), "-o", o], check=True,
                   capture_output=True)
subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out_dir, "libhuffman_amd.so")]
               + objs, check=True)
print(out_dir)
