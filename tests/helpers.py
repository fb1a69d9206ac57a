"""Shared comparison helpers for the parity tests."""
import numpy as np

# Tolerance of the north star: hom_conf / het_conf within 1e-10 relative of
# the reference.  Below DBL_MIN the reference's own result is a denormal with
# fewer significant bits, so there the bound is absolute: 64 denormal ulps.
REL_TOL = 1e-10
DENORM_ABS = 64 * 4.9406564584124654e-324


def conf_mismatch(a, b):
    """Boolean mask of confidences that violate the tolerance (NaN == NaN with
    the same sign bit, infinities exact)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    nan_a, nan_b = np.isnan(a), np.isnan(b)
    bad = nan_a != nan_b
    both = nan_a & nan_b
    bad |= both & (np.signbit(a) != np.signbit(b))
    fin = ~(nan_a | nan_b)
    eq = fin & (a == b)
    diff = np.abs(a - b, where=fin & ~eq, out=np.zeros_like(a))
    tol = np.maximum(REL_TOL * np.abs(b), DENORM_ABS)
    bad |= fin & ~eq & ~(diff <= tol)
    return bad


def assert_parity(code, hom, het, rcode, rhom, rhet, what=""):
    code = np.asarray(code)
    rcode = np.asarray(rcode)
    bad_code = code != rcode
    bh, bt = conf_mismatch(hom, rhom), conf_mismatch(het, rhet)
    if bad_code.any() or bh.any() or bt.any():
        i = int(np.flatnonzero(bad_code | bh | bt)[0])
        raise AssertionError(
            f"{what}: {int(bad_code.sum())} code / {int(bh.sum())} hom / {int(bt.sum())} het "
            f"mismatches; first at {i}: code {code[i]:#x} vs {rcode[i]:#x}, "
            f"hom {hom[i]!r} vs {rhom[i]!r}, het {het[i]!r} vs {rhet[i]!r}")


def all_profiles(cmax):
    """Every (A,C,G,T) with A+C+G+T <= cmax."""
    r = np.arange(cmax + 1)
    a, c, g, t = np.meshgrid(r, r, r, r, indexing="ij")
    m = (a + c + g + t) <= cmax
    return np.stack([a[m], c[m], g[m], t[m]], axis=1).astype(np.uint16)
