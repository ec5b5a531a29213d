"""Latency of the codebook and header stages, device against host.

For a Zipf(1.1) histogram of a 1 GiB device stream scaled x16 (the 16 GiB bench
stream's shape, U = 65 536) and a uniform one: the device codebook
(hz_codebook_build_device), device header writer and device header parser, each
timed as launch -> stream sync (wall) and by HIP events on the library's stream;
against the host builder / writer / parser (hz_codebook_build, hz_header_write,
hz_header_parse) plus the copies the host path needs (histogram D2H, codebook H2D).
Median of --reps. Writes one JSON object to --out."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import huffman_amd as hz  # noqa: E402
from huffman_amd._lib import Codebook  # noqa: E402
from huffman_amd.pipeline import StreamCodec  # noqa: E402


def med(xs):
    return float(np.median(xs))


def timed(c, fn, reps):
    wall, ev = [], []
    for _ in range(reps):
        c.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        fn()
        e1.record()
        c.sync()
        t1 = time.perf_counter()
        wall.append((t1 - t0) * 1e3)
        ev.append(e0.elapsed_time(e1))
    return {"wall_ms": med(wall), "device_ms": med(ev)}


def host_timed(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return med(ts)


def case(c, kind, reps):
    n = 1 << 30
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    c.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=42)
    c.histogram(x)
    c.sync()
    del x
    h = c.hist.cpu().numpy().view(np.uint64) * np.uint64(16)
    hd = torch.from_numpy(h.view(np.int64)).cuda()
    n16 = 16 << 30
    d_cb = torch.zeros(ctypes.sizeof(Codebook), dtype=torch.uint8, device="cuda")
    out = {"U": int((h > 0).sum())}
    out["device_codebook"] = timed(c, lambda: c.dev.codebook_build(hd.data_ptr(), d_cb.data_ptr()), reps)
    cb_dev = Codebook.from_buffer_copy(d_cb.cpu().numpy().tobytes())
    cb = hz.build_codebook(h)
    same = all(bytes(getattr(cb_dev, f)) == bytes(getattr(cb, f)) for f in ("order", "len", "code"))
    out["device_codebook_equals_host"] = bool(same and cb_dev.max_len == cb.max_len)
    out["host_codebook_ms"] = host_timed(lambda: hz.build_codebook(h), reps)
    out["host_hist_d2h_ms"] = host_timed(lambda: c.hist.cpu(), reps)
    pin = torch.empty(ctypes.sizeof(Codebook), dtype=torch.uint8).pin_memory()
    pin.numpy()[:] = np.frombuffer(bytes(cb), dtype=np.uint8)
    out["codebook_h2d"] = timed(c, lambda: d_cb.copy_(pin, non_blocking=True), reps)
    cap = 16 + 65536 * 11
    hout = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    info = torch.zeros(6, dtype=torch.int64, device="cuda")
    out["device_header_write"] = timed(
        c, lambda: c.dev.header_write(d_cb.data_ptr(), n16, 0, hout.data_ptr(), cap, info.data_ptr()), reps)
    out["host_header_write_ms"] = host_timed(lambda: hz.write_header(cb, n16, 0), reps)
    head, pbits, pend = hz.write_header(cb, n16, 0)
    blob = head + (bytes([pend]) if pbits else b"") + bytes(64)
    f = torch.from_numpy(np.frombuffer(blob, dtype=np.uint8).copy()).cuda()
    out["header_bytes"] = len(head)
    out["device_header_parse"] = timed(
        c, lambda: c.dev.header_parse(f.data_ptr(), len(blob), d_cb.data_ptr(), info.data_ptr()), reps)
    cb_p = Codebook.from_buffer_copy(d_cb.cpu().numpy().tobytes())
    out["device_parse_equals_host_codebook"] = all(
        bytes(getattr(cb_p, k)) == bytes(getattr(cb, k)) for k in ("order", "len", "code"))
    out["host_header_parse_ms"] = host_timed(lambda: hz.parse_header(blob), reps)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=21)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    c = StreamCodec(0)
    res = {"note": "wall = launch -> stream sync on the host; device = HIP events around the launches",
           "zipf_16gib_shape": case(c, 1, a.reps), "uniform_16gib_shape": case(c, 0, a.reps)}
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
