"""Host write bandwidth into one page-cached file (the CLIs' fwrite bound): one write(),
8-thread pwrite, and 8-thread memcpy into a shared mmap of the file.
usage: python tools/debug/write_bw.py [GiB] [dir]"""
import mmap
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 4
d = sys.argv[2] if len(sys.argv) > 2 else (os.environ.get("TMPDIR") or "/tmp")
n = int(gib * (1 << 30))
src = np.random.default_rng(0).integers(0, 255, size=n, dtype=np.uint8)
T = 8


def run(name, fn):
    fd, path = tempfile.mkstemp(dir=d)
    os.close(fd)
    t0 = time.perf_counter()
    fn(path)
    dt = time.perf_counter() - t0
    os.remove(path)
    print(f"{name}: {n / dt / 1e9:.2f} GB/s ({dt:.2f} s)", flush=True)


def single(path):
    with open(path, "wb") as f:
        f.write(memoryview(src))


def pw(path):
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    piece = (n + T - 1) // T
    mv = memoryview(src)
    with ThreadPoolExecutor(T) as ex:
        list(ex.map(lambda i: os.pwrite(fd, mv[i * piece:(i + 1) * piece], i * piece), range(T)))
    os.close(fd)


def mm(path):
    fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
    os.ftruncate(fd, n)
    m = mmap.mmap(fd, n, mmap.MAP_SHARED, mmap.PROT_WRITE)
    dst = np.frombuffer(m, dtype=np.uint8)
    piece = (n + T - 1) // T
    with ThreadPoolExecutor(T) as ex:
        list(ex.map(lambda i: np.copyto(dst[i * piece:(i + 1) * piece], src[i * piece:(i + 1) * piece]), range(T)))
    del dst
    m.close()
    os.close(fd)


print(f"dir {d}, {gib} GiB, statfs type {os.statvfs(d).f_fsid if hasattr(os.statvfs(d), 'f_fsid') else '?'}")
for name, fn in [("write", single), ("pwrite x8", pw), ("mmap x8", mm), ("write", single), ("pwrite x8", pw),
                 ("mmap x8", mm)]:
    run(name, fn)
