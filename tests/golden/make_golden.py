"""Regenerate the golden fixtures in tests/golden/ (run in the build container,
where /root/reference exists; the fixtures themselves are committed).

Fixtures (data only -- no reference source is copied):
  romeo.txt                         the reference's own test input (reference Makefile:17-29)
  romeo.txt.baseline.compressed     output of the reference baseline encoder
                                    (baseline/Compressor.cu, built by oracle/Makefile)
  romeo.txt.compressed              the expected output of THIS build's encoder
                                    (Compressor.cu semantics, oracle/hz_oracle.c), accepted
                                    by the reference decoder (Decompressor.cu)
  pexels-vlad-alexandru-popa-1402787.jpg   the reference's second data file (U = 65 289)
  synth_*.bin (+ .baseline.compressed, .compressed)  small generator streams
  kat.json                          hand-derived codebook KAT of SURVEY.md 8(a4)
  MANIFEST.json                     sha256 of every fixture
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402

REF = "/root/reference"


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def baseline_compress(src, dst):
    exe = oracle_lib.ref_binary("archive_baseline")
    with tempfile.TemporaryDirectory() as td:
        t = os.path.join(td, "in")
        shutil.copy(src, t)
        subprocess.run([exe, "in"], cwd=td, check=True, capture_output=True)
        shutil.copy(os.path.join(td, "in.compressed"), dst)


def ref_decodes(comp, original):
    exe = oracle_lib.ref_binary("extract")
    with tempfile.TemporaryDirectory() as td:
        shutil.copy(comp, os.path.join(td, "x.compressed"))
        subprocess.run([exe, "x.compressed"], cwd=td, check=True, capture_output=True)
        with open(os.path.join(td, "DECOMPRESSED_FILE"), "rb") as f:
            got = f.read()
    with open(original, "rb") as f:
        return got == f.read()


def copy_data(name):
    dst = os.path.join(HERE, name)
    if os.path.exists(dst):
        os.chmod(dst, 0o644)
    shutil.copyfile(os.path.join(REF, name), dst)


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all", "ref"], check=True)
    copy_data("romeo.txt")
    copy_data("pexels-vlad-alexandru-popa-1402787.jpg")
    inputs = ["romeo.txt"]
    for name, n, kind in [("synth_zipf_65537.bin", 65537, 1), ("synth_unif_65536.bin", 65536, 0),
                          ("synth_zipf_4099.bin", 4099, 1)]:
        oracle_lib.generate(n, offset=0, kind=kind, seed=42).tofile(os.path.join(HERE, name))
        inputs.append(name)
    for name in inputs:
        src = os.path.join(HERE, name)
        baseline_compress(src, src + ".baseline.compressed")
        with open(src, "rb") as f:
            enc = oracle_lib.encode(f.read())
        with open(src + ".compressed", "wb") as f:
            f.write(enc)
        assert ref_decodes(src + ".compressed", src), name
        assert ref_decodes(src + ".baseline.compressed", src), name
    kat = {
        "source": "SURVEY.md 8(a4); leaves in sorted order a=1,b=1,c=1,d=1,e=2",
        "freqs": [1, 1, 1, 1, 2],
        "gpu_codes": ["001", "000", "11", "10", "01"],
        "baseline_codes": ["011", "010", "001", "000", "1"],
    }
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    manifest = {n: sha(os.path.join(HERE, n)) for n in sorted(os.listdir(HERE))
                if not n.endswith(".py") and n != "MANIFEST.json"}
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
