"""The product's host code -- parse.cpp (sid_parse_text), emit.cpp
(sid_format_csv, sid_format_double) and fmt.h's host build of the device %g
-- compiled with AddressSanitizer + UndefinedBehaviorSanitizer
(tests/asan) and run over the parser's fuzz corpus, the golden
pileups and the formatter's hard doubles.  A sanitizer report fails the test,
and every output must equal the unsanitized build/libsid.so's.  CPU only."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from test_emit import sample_doubles
from test_fmt import boundary_values, tie_values
from test_parser import blank, fuzz_lines, product_line

HERE = os.path.dirname(os.path.abspath(__file__))
ASAN = os.path.join(HERE, "asan", "_build", "sid_asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def asan():
    if not shutil.which("make") or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc / make")
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "asan")], check=True)
    return ASAN


def run(asan, *args):
    r = subprocess.run([asan] + list(args), capture_output=True, env=ENV, timeout=600)
    err = r.stderr.decode(errors="replace")
    assert "AddressSanitizer" not in err and "runtime error" not in err and "LeakSanitizer" not in err, err[-3000:]
    assert r.returncode == 0, err[-3000:]
    return r.stdout


def expected_line(sid, line):
    got = product_line(sid, line)
    if got is None:
        return b"NONE"
    if got[0] == "ERR":
        return b"ERR\t%d" % {"std::invalid_argument": 4, "std::logic_error": 6}[got[1]]
    return ("OK\t%s\t%d\t%d\t%d\t%d\t%d" % (got[1], got[2], *got[3:])).encode("latin-1")


def test_parser_fuzz_sanitized(sid, asan, tmp_path):
    lines = [l for s in (1, 2, 3) for l in fuzz_lines(s, 1500) if b"\n" not in l and not blank(l)]
    gold = open(os.path.join(HERE, "golden", "edge.plp"), "rb").read().split(b"\n")
    lines += [l for l in gold if l and not blank(l)]
    p = tmp_path / "lines.txt"
    p.write_bytes(b"\n".join(lines) + b"\n")
    out = run(asan, "lines", str(p)).split(b"\n")[:-1]
    assert len(out) == len(lines)
    for line, got in zip(lines, out):
        assert got == expected_line(sid, line), line


def synth_arrays(n):
    i = np.arange(n, dtype=np.uint64)
    code = ((i * 37) & 0x0F).astype(np.uint8)
    code |= np.where(i % 5 == 0, 0x80, 0).astype(np.uint8)
    code |= np.where(i % 11 == 3, 0x40, 0).astype(np.uint8)
    hom = np.ldexp(((i * 2654435761) % 1000003).astype(np.float64) / 1000003.0, -(i % 60).astype(np.int64))
    het = np.ldexp(((i * 40503 + 7) % 999983).astype(np.float64) / 999983.0, -(i % 1075).astype(np.int64))
    return code, hom, het


@pytest.mark.parametrize("name,threads", [("c1", 1), ("c1", 4), ("edge", 3), ("deep", 8), ("long", 2)])
def test_parse_and_csv_sanitized(sid, asan, tmp_path, name, threads):
    if name in ("c1", "edge"):
        text = open(os.path.join(HERE, "golden", {"c1": "c1_10k.plp", "edge": "edge.plp"}[name]), "rb").read()
    elif name == "deep":
        text = sid.synth_text(5, 3000, 200.0, sites_per_chrom=1000)
    else:   # chrom names past any fixed buffer
        text = b"".join(b"scaffold_%d_%s\t%d\tA\t2\t.,\tII\n" % (k, b"x" * (k % 90), k + 1) for k in range(2000))
    p = tmp_path / "in.plp"
    p.write_bytes(text)
    got = run(asan, "csv", str(p), str(threads))
    s = sid.parse_text(text)
    code, hom, het = synth_arrays(len(s))
    assert got == sid.format_csv(s, code, hom, het, "p_value")


def test_g6_sanitized(sid, asan, tmp_path):
    vals = np.concatenate([sample_doubles(20_000), tie_values(), boundary_values()])
    p = tmp_path / "v.f64"
    vals.astype(np.float64).tofile(p)
    out = run(asan, "g6", str(p)).split(b"\n")[:-1]
    assert len(out) == len(vals)
    for v, line in zip(vals, out):
        a, b = line.split(b"\t")
        try:
            want = sid.format_g6(float(v)).encode()
        except sid.SidError:
            want = b"RANGE"
        assert a == want, v
        assert b == sid.format_double(float(v)).encode(), v
