"""Host write bandwidth into one file (the CLIs' fwrite bound): one write(), 8-thread
pwrite, 8-thread memcpy into a shared mmap, pwrite after fallocate, and O_DIRECT pwrite
(page-aligned source, 8 threads, 64 MiB pieces).
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


def fpw(path):
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    os.posix_fallocate(fd, 0, n)
    piece = (n + T - 1) // T
    mv = memoryview(src)
    with ThreadPoolExecutor(T) as ex:
        list(ex.map(lambda i: os.pwrite(fd, mv[i * piece:(i + 1) * piece], i * piece), range(T)))
    os.close(fd)


asrc = np.frombuffer(mmap.mmap(-1, n), dtype=np.uint8)  # page aligned
asrc[:] = src


def direct(path):
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | os.O_DIRECT, 0o644)
    P = 64 << 20
    mv = memoryview(asrc)
    offs = list(range(0, n - n % P, P))
    with ThreadPoolExecutor(T) as ex:
        list(ex.map(lambda o: os.pwrite(fd, mv[o:o + P], o), offs))
    os.close(fd)


def fs_of(d):
    best = ("?", "")
    for line in open("/proc/mounts"):
        f = line.split()
        if os.path.realpath(d).startswith(f[1]) and len(f[1]) >= len(best[1]):
            best = (f[2], f[1])
    return best


print("filesystem", fs_of(d), flush=True)
for name, fn in [("fallocate+pwrite x8", fpw), ("O_DIRECT pwrite x8", direct), ("O_DIRECT pwrite x8", direct)]:
    try:
        run(name, fn)
    except OSError as e:
        print(name, "failed:", e, flush=True)
print(f"dir {d}, {gib} GiB, statfs type {os.statvfs(d).f_fsid if hasattr(os.statvfs(d), 'f_fsid') else '?'}")
for name, fn in [("write", single), ("pwrite x8", pw), ("mmap x8", mm), ("write", single), ("pwrite x8", pw),
                 ("mmap x8", mm)]:
    run(name, fn)
