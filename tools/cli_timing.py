"""Stage split of the drop-in CLIs on a real file.

Writes a synthetic Zipf(1.1) file of --gib GiB (the bench's generator, seed 42),
runs bin/archive and bin/extract on it with HZ_TIMING=1 (one JSON stage line
each on stderr: fread, fwrite, host, H2D, kernels, D2H, total), checks that
DECOMPRESSED_FILE equals the input, and prints one JSON line.

usage: python tools/cli_timing.py [--gib 4] [--dir DIR] [--out profiles/xxx.json]
"""
import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[cli_timing {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def pick_dir(want_bytes, override):
    if override:
        return override
    for d in (os.environ.get("TMPDIR"), "/tmp", ROOT):
        if d and os.path.isdir(d) and shutil.disk_usage(d).free > want_bytes:
            return d
    raise SystemExit(f"no directory with {want_bytes / 2**30:.1f} GiB free")


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        while True:
            b = f.read(64 << 20)
            if not b:
                return h.hexdigest()
            h.update(b)


def run_cli(exe, arg, cwd):
    env = dict(os.environ, HZ_TIMING="1")
    t0 = time.perf_counter()
    r = subprocess.run([exe, arg], cwd=cwd, env=env, capture_output=True, text=True, timeout=600)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise SystemExit(f"{exe} failed ({r.returncode}): {r.stdout[-400:]} {r.stderr[-400:]}")
    stages = [json.loads(l) for l in r.stderr.splitlines() if l.startswith("{")]
    return wall, stages[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    n = int(args.gib * (1 << 30)) | 1  # odd: the last byte travels in the header
    work = os.path.join(pick_dir(3 * n + (1 << 30), args.dir), f"hz_cli_{os.getpid()}")
    os.makedirs(work, exist_ok=True)
    src = os.path.join(work, "input.bin")
    try:
        import torch
        from huffman_amd.pipeline import StreamCodec
        codec = StreamCodec(0)
        step = 1 << 30
        t0 = time.perf_counter()
        with open(src, "wb") as f:
            buf = torch.empty(step, dtype=torch.uint8, device="cuda")
            for off in range(0, n, step):
                m = min(step, n - off)
                codec.dev.generate(buf.data_ptr(), m, offset=off, kind=1, alpha=1.1, seed=42)
                codec.sync()
                f.write(buf[:m].cpu().numpy().tobytes())
            del buf
        log(f"wrote {n} bytes in {time.perf_counter() - t0:.1f} s to {src}")
        want = sha(src)
        bindir = os.path.join(ROOT, "huffman_amd", "bin")
        a_wall, a_st = run_cli(os.path.join(bindir, "archive"), src, work)
        log(f"archive {a_wall:.2f} s: {a_st}")
        comp = src + ".compressed"
        csize = os.path.getsize(comp)
        e_wall, e_st = run_cli(os.path.join(bindir, "extract"), comp, work)
        log(f"extract {e_wall:.2f} s: {e_st}")
        ok = sha(os.path.join(work, "DECOMPRESSED_FILE")) == want
        line = {
            "file_bytes": n, "compressed_bytes": csize, "data": "synthetic Zipf(1.1) bytes, seed 42",
            "round_trip_identical": ok,
            "archive": dict(a_st, process_wall_s=round(a_wall, 3), GBps_of_input=round(n / a_wall / 1e9, 3)),
            "extract": dict(e_st, process_wall_s=round(e_wall, 3), GBps_of_output=round(n / e_wall / 1e9, 3)),
            "note": "stage times are busy times; host file I/O overlaps device copies and kernels",
        }
        print(json.dumps(line), flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(line, f, indent=1)
        if not ok:
            raise SystemExit("round trip differs")
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
