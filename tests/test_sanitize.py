"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer.

The native ingest (waafle_amd/csrc/wf_ingest.cpp: a multi-threaded parser of untrusted
text) is compiled from source with -fsanitize=address,undefined into a standalone driver
(tests/sanitize/ingest_driver.cpp) and run on the demo inputs, seeded synthetic inputs
and malformed variants, with 1, 3 and 8 threads; every run must be clean (any report
aborts the driver) and all thread counts must give the same arrays.
(The C-ABI of libwaafle_hip, wf_api.cpp, is host code that drives the GPU: its sanitizer
run is tests/sanitize/api_driver.cpp, built and run on the GPU box by scripts/gpu_r2.sh.)
"""
import os
import shutil
import subprocess

import pytest

import golden_cases as gc
from waafle_amd import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "waafle_amd", "csrc", "wf_ingest.cpp")
DRIVER = os.path.join(REPO, "tests", "sanitize", "ingest_driver.cpp")


@pytest.fixture(scope="module")
def asan_driver(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = str(tmp_path_factory.mktemp("asan") / "ingest_asan")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I" + os.path.join(REPO, "include"), SRC, DRIVER, "-o", out]
    subprocess.run(cmd, check=True)
    return out


def run(driver, paths, mgl="200", threads=("1", "3", "8")):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([driver] + list(paths) + [mgl] + list(threads), capture_output=True,
                       text=True, env=env, timeout=300)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    assert r.returncode in (0,), (r.returncode, r.stdout, r.stderr[-2000:])
    return r.stdout.splitlines()


def same_hash(lines):
    hashes = {l.split("hash=")[1] for l in lines if "hash=" in l}
    return len(hashes) == 1


def test_ingest_asan_demo(asan_driver, tmp_path):
    paths = [gc.demo_file(f, tmp_path) for f in gc.DEMO_FILES["prodigal"]][:3]
    out = run(asan_driver, paths)
    assert len(out) == 4 and same_hash(out)


def test_ingest_asan_synthetic(asan_driver, tmp_path):
    data = synth.generate(n=2000, genes=8, clades=200, seed=3, short_frac=0.2)
    fna, blast, gff, _ = synth.write_text(data, str(tmp_path), "s")
    out = run(asan_driver, [fna, blast, gff], mgl="100")
    assert len(out) == 4 and same_hash(out) and "hits=" in out[0]


def test_ingest_asan_malformed(asan_driver, tmp_path):
    data = synth.generate(n=50, genes=4, clades=20, seed=4, decoys=2)
    fna, blast, gff, _ = synth.write_text(data, str(tmp_path), "m")
    text = open(blast).read().splitlines()
    variants = {
        "short_row": text[:5] + ["contig1\tx"] + text[5:],
        "bad_float": text[:3] + [text[3].replace("\t0\t0.0\t", "\t0\tx.5\t")] + text[4:],
        "no_newline": text[:-1] + [text[-1]],
        "crlf": [l + "\r" for l in text],
        "huge_int": text[:2] + [text[2].replace("\t", "\t99999999999999999999", 1)] + text[3:],
        "empty": [],
    }
    for name, rows in variants.items():
        p = tmp_path / (name + ".blastout")
        body = "\n".join(rows)
        p.write_text(body if name == "no_newline" else body + ("\n" if rows else ""))
        run(asan_driver, [fna, str(p), gff])             # clean run: parsed or fallback
    bad_fna = tmp_path / "bad.fna"
    bad_fna.write_text(">a\nNNN\n\n>b\nNN\n")
    run(asan_driver, [str(bad_fna), blast, gff])
