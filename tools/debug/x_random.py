"""Debug: replay test_gpu_extract.py::test_indexless_random_streams up to case K and report, for each
case, whether the file decodes (hz_decode_host, index-less); for a failing case the codebook, the
payload geometry and the mismatching symbol indices with their stream bits (CPU oracle walk).
usage: python tools/debug/x_random.py [K] [SEG_LEAD values to retry ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import oracle_lib  # noqa: E402
import huffman_amd as hz  # noqa: E402
from test_gpu_extract import _random_stream  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 24
rng = np.random.default_rng(20261018)
for case in range(K):
    data, what = _random_stream(rng)
    if data.size >= 2:
        rng.integers(0, 48)
    blob = oracle_lib.encode(data)
    got = hz.decode(blob)
    ok = got == data.tobytes()
    print(case, what, "ok" if ok else "MISMATCH", flush=True)
    if ok:
        continue
    g = np.frombuffer(got, dtype=np.uint8)
    bad = np.nonzero(g[: data.size] != data)[0]
    sym_bad = np.unique(bad // 2)
    hist = oracle_lib.hist16(data)
    order, ln, code = oracle_lib.codebook(hist)
    info = hz.parse_header(np.frombuffer(blob, dtype=np.uint8))[1] if hasattr(hz, "parse_header") else None
    print("  codebook U", order.size, "lens", sorted(set(int(ln[s]) for s in order)), flush=True)
    for s in order[:8]:
        print("   sym %5d count %10d len %2d code %s" % (s, hist[s], ln[s], format(int(code[s]), "b").zfill(int(ln[s]))))
    print("  bad symbols", sym_bad.size, "first", sym_bad[:20].tolist(), "last", sym_bad[-5:].tolist(), flush=True)
    # stream bits of the symbols around the first bad one (CPU oracle walk from the payload start)
    pay = np.frombuffer(blob, dtype=np.uint8)
    if info is not None:
        start = int(info.payload_byte) * 8 + int(info.payload_bit)
        print("  payload_byte", info.payload_byte, "payload_bit", info.payload_bit, "nsym", info.n // 2,
              "payload bits", pay.size * 8 - start, flush=True)
        s0 = int(sym_bad[0])
        n_before, bit_at, _ = oracle_lib.walk(pay, ln, code, start, pay.size * 8, max_count=s0)
        print("  first bad symbol %d starts at stream bit %d (payload bit %d)" % (s0, bit_at, bit_at - start))
        print("  expected", data[2 * s0: 2 * s0 + 16].tolist(), "\n  got     ", list(g[2 * s0: 2 * s0 + 16]))
    for lead in sys.argv[2:]:
        code_s = ("import sys, numpy as np; sys.path.insert(0, %r); import huffman_amd as hz; "
                  "b = open('/tmp/xr_blob', 'rb').read(); d = open('/tmp/xr_data', 'rb').read(); "
                  "print('lead', %r, hz.decode(b) == d)") % (ROOT, lead)
        open("/tmp/xr_blob", "wb").write(blob)
        open("/tmp/xr_data", "wb").write(data.tobytes())
        r = subprocess.run([sys.executable, "-c", code_s], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, HZ_SEG_LEAD=lead))
        print("  ", r.stdout.strip(), r.stderr.strip()[-300:], flush=True)
