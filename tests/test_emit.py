"""CSV emitter (emit.cpp) against the reference's iostream formatting
(call.hpp:29-38: default ostream<<double == printf("%g"), precision 6).  CPU."""
import ctypes as C
import struct

import numpy as np

libc = C.CDLL("libc.so.6")
libc.snprintf.restype = C.c_int


def printf_g(v: float) -> str:
    buf = C.create_string_buffer(64)
    libc.snprintf(buf, 64, b"%g", C.c_double(v))
    return buf.value.decode()


def sample_doubles(n=200_000, seed=0):
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2**63, size=n, dtype=np.int64).view(np.float64)
    parts = [
        bits,
        rng.random(n),
        np.exp(-rng.random(n) * 750.0),                          # p-value like, down to denormals
        np.array([0.0, -0.0, 1.0, -1.0, float("inf"), float("-inf"), float("nan"),
                  -float("nan"), 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308,
                  0.0001, 0.00001, 999999.5, 9999995.0, 0.095891, 4.5561e-07, 1e16, 123456789.0]),
        np.nextafter(np.array([1e-5, 1e-4, 1.0, 10.0, 1e5, 1e6]), 0),
    ]
    return np.concatenate(parts)


def test_format_double_matches_printf(sid):
    vals = sample_doubles()
    bad = []
    for v in vals:
        a, b = sid.format_double(float(v)), printf_g(float(v))
        if a != b:
            bad.append((float(v), a, b))
            if len(bad) > 5:
                break
    assert not bad, bad


def test_negative_nan_prints_minus_nan(sid):
    neg_nan = struct.unpack("<d", struct.pack("<Q", 0xFFF8000000000000))[0]
    assert sid.format_double(neg_nan) == printf_g(neg_nan) == "-nan"


def test_format_csv_records(sid):
    text = sid.synth_text(5, 5000, 30.0, sites_per_chrom=1700)
    s = sid.parse_text(text)
    rng = np.random.default_rng(1)
    n = len(s)
    code = rng.integers(0, 256, size=n).astype(np.uint8)
    hom = np.where(rng.random(n) < 0.5, 1.0, rng.random(n) ** 20)
    het = np.where(rng.random(n) < 0.5, 1.0, rng.random(n) ** 40)
    for conf_type in ("p_value", "probability"):
        out = sid.format_csv(s, code, hom, het, conf_type)
        want = []
        for i in range(n):
            if code[i] & 0x40:
                continue
            name = [nm for st, nm in s.chroms if st <= i][-1].decode()
            c = int(code[i])
            want.append(f"{name},{s.positions[i]},{'het' if c & 0x80 else 'hom'},"
                        f"{'ACGT'[c & 3]}{'ACGT'[(c >> 2) & 3]},{printf_g(hom[i])},{printf_g(het[i])},{conf_type}\n")
        assert out.decode() == "".join(want)
