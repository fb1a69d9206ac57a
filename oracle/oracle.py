"""ctypes wrapper of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / baseline, never as the
thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
CLI = os.path.join(HERE, "_build", "sid_oracle")
REF_PILEUP = os.path.join(HERE, "_ref", "ref_pileup")

_L = None


class Est(C.Structure):
    _fields_ = [("heterozygosity", C.c_double), ("error_rate", C.c_double), ("fval", C.c_double),
                ("iterations", C.c_int), ("converged", C.c_int), ("status", C.c_int),
                ("evaluations", C.c_size_t)]


class Profile(C.Structure):
    _fields_ = [("profile", C.c_uint16 * 4), ("count", C.c_uint32), ("coverage", C.c_uint32)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.c_void_p
        L.oracle_gsl_chisq_Q.restype = C.c_double
        L.oracle_gsl_chisq_Q.argtypes = [C.c_double]
        L.oracle_gsl_lngamma.restype = C.c_double
        L.oracle_gsl_lngamma.argtypes = [C.c_double]
        L.oracle_call_local.restype = None
        L.oracle_call_local.argtypes = [P, C.c_size_t, C.c_double, C.c_double, C.c_double, P, P, P]
        L.oracle_call_method.restype = C.c_int
        L.oracle_call_method.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, P,
                                         C.c_size_t, P, P, P, C.POINTER(Est), C.POINTER(C.c_size_t),
                                         C.c_int]
        L.oracle_read_bases.restype = None
        L.oracle_read_bases.argtypes = [C.c_char_p, C.c_char, P]
        L.oracle_parse_qualities.restype = C.c_int
        L.oracle_parse_qualities.argtypes = [C.c_char_p, P, C.c_int]
        L.oracle_count_unique.restype = C.c_size_t
        L.oracle_count_unique.argtypes = [P, C.c_size_t, C.POINTER(C.POINTER(Profile))]
        L.oracle_nucleotide_distribution.restype = None
        L.oracle_nucleotide_distribution.argtypes = [C.POINTER(Profile), C.c_size_t, P]
        L.oracle_compound_likelihood.restype = C.c_double
        L.oracle_compound_likelihood.argtypes = [C.POINTER(Profile), C.c_size_t, P, C.c_double,
                                                 C.c_double]
        L.oracle_filter_min_coverage.restype = C.c_size_t
        L.oracle_filter_min_coverage.argtypes = [C.POINTER(Profile), C.c_size_t]
        L.oracle_read_bases_seq.restype = C.c_int
        L.oracle_read_bases_seq.argtypes = [C.c_char_p, C.c_char, C.c_char_p, C.c_int]
        L.oracle_call_quality_text.restype = C.c_int
        L.oracle_call_quality_text.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_double, C.c_double, P, P, P,
                                               C.c_size_t, C.POINTER(C.c_size_t), C.c_int]
        _L = L
    return _L


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def chisq_Q(x: float) -> float:
    return lib().oracle_gsl_chisq_Q(float(x))


def lngamma(x: float) -> float:
    return lib().oracle_gsl_lngamma(float(x))


def call_local(counts: np.ndarray, snp_prior=-1.0, site_error_threshold=0.1, significance_level=0.05):
    counts = np.ascontiguousarray(counts, np.uint16).reshape(-1, 4)
    n = len(counts)
    code = np.zeros(n, np.uint8)
    h = np.zeros(n, np.float64)
    t = np.zeros(n, np.float64)
    lib().oracle_call_local(_p(counts), n, snp_prior, site_error_threshold, significance_level,
                            _p(code), _p(h), _p(t))
    return code, h, t


METHOD = {"local": 0, "likelihood_ratio": 1, "bayes": 2}


def call_method(counts: np.ndarray, method="local", estimate_prior=False, snp_prior=-1.0,
                site_error_threshold=0.1, significance_level=0.05, verbose=False):
    """Whole method as the reference runs it (dedupe, estimate, BH ...).
    Returns (rc, code, hom, het, Est, n_unique)."""
    counts = np.ascontiguousarray(counts, np.uint16).reshape(-1, 4)
    n = len(counts)
    code = np.zeros(max(n, 1), np.uint8)
    h = np.zeros(max(n, 1), np.float64)
    t = np.zeros(max(n, 1), np.float64)
    est = Est()
    u = C.c_size_t(0)
    rc = lib().oracle_call_method(METHOD[method], int(estimate_prior), snp_prior,
                                  site_error_threshold, significance_level, _p(counts), n, _p(code),
                                  _p(h), _p(t), C.byref(est), C.byref(u), int(verbose))
    return rc, code[:n], h[:n], t[:n], est, u.value


def read_bases_seq(s: bytes, ref: bytes) -> bytes:
    """pileup.cpp:70-153 bases vector (upper case, read order)."""
    n = lib().oracle_read_bases_seq(s, ref, None, 0)
    buf = C.create_string_buffer(max(n, 1))
    lib().oracle_read_bases_seq(s, ref, buf, n)
    return buf.raw[:n]


def call_quality(text: bytes, estimate_prior=False, snp_prior=-1.0, significance_level=0.05):
    """call.cpp:291-372 over a pileup text (7 fields).  Returns (rc, code, hom, het):
    rc = 0, or 1 malformed / 2 missing mapping qualities / 3 no chromosome /
    4 no base qualities (the first bad line), or 10 + the -R estimate's rc."""
    n = C.c_size_t(0)
    L = lib()
    rc = L.oracle_call_quality_text(text, len(text), int(estimate_prior), snp_prior, significance_level,
                                    None, None, None, 0, C.byref(n), 0)
    if rc:
        return rc, None, None, None
    m = n.value
    code = np.zeros(max(m, 1), np.uint8)
    h = np.zeros(max(m, 1), np.float64)
    t = np.zeros(max(m, 1), np.float64)
    rc = L.oracle_call_quality_text(text, len(text), int(estimate_prior), snp_prior, significance_level, _p(code),
                                    _p(h), _p(t), m, C.byref(n), 0)
    return rc, code[:m], h[:m], t[:m]


def read_bases(s: bytes, ref: bytes) -> np.ndarray:
    out = np.zeros(4, np.uint16)
    lib().oracle_read_bases(s, ref, _p(out))
    return out


def unique_profiles(counts: np.ndarray, min_coverage4=False):
    counts = np.ascontiguousarray(counts, np.uint16).reshape(-1, 4)
    ptr = C.POINTER(Profile)()
    u = lib().oracle_count_unique(_p(counts), len(counts), C.byref(ptr))
    if min_coverage4 and u:
        u = lib().oracle_filter_min_coverage(ptr, u)
    rows = [(tuple(ptr[i].profile), ptr[i].count, ptr[i].coverage) for i in range(u)]
    return rows, ptr, u


def distribution(counts: np.ndarray, min_coverage4=True):
    rows, ptr, u = unique_profiles(counts, min_coverage4)
    d = np.zeros(4, np.float64)
    lib().oracle_nucleotide_distribution(ptr, u, _p(d))
    return d


def compound_likelihood(counts: np.ndarray, pi: float, eps: float):
    rows, ptr, u = unique_profiles(counts, True)
    d = np.zeros(4, np.float64)
    lib().oracle_nucleotide_distribution(ptr, u, _p(d))
    return lib().oracle_compound_likelihood(ptr, u, _p(d), pi, eps)


def run_cli(args, **kw):
    """Run the oracle CLI (reference sid.cpp restated)."""
    if not os.path.exists(CLI):
        build()
    return subprocess.run([CLI] + list(args), capture_output=True, **kw)


def ref_pileup_available() -> bool:
    return os.path.exists(REF_PILEUP)


def ref_pileup(mode: str, data: bytes) -> bytes:
    """Drive the REFERENCE's pileup.cpp (oracle/_ref), see ref_pileup_harness.cpp."""
    return subprocess.run([REF_PILEUP, mode], input=data, capture_output=True, check=True).stdout
