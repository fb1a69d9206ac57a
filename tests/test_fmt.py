"""The device CSV formatter's %g (fmt.h: exact six significant digits by
multi-limb integer arithmetic, rounded half-to-even) -- its host build against
printf("%g") and std::to_chars, which the reference's operator<<(double)
matches (call.hpp:29-38).  CPU; the device build is compared with the same
values in tests/test_textpath_gpu.py."""
import numpy as np

from test_emit import printf_g, sample_doubles


def tie_values():
    """Dyadic rationals whose exact decimal has exactly 7 significant digits
    ending in 5: %g must round them half-to-even (e.g. 13/128 = 0.1015625)."""
    out = []
    for den_pow in range(1, 30):
        den = 2 ** den_pow
        for num in range(1, 2000, 2):
            v = num / den
            d = f"{v:.30e}".split("e")[0].replace(".", "").rstrip("0")
            if len(d) == 7 and d.endswith("5"):
                out.append(v)
    # and scaled by powers of ten that keep them exact
    more = [v * 10 ** k for v in out[:200] for k in range(0, 4) if float(v * 10 ** k) < 2 ** 53]
    return np.array(out + more, dtype=np.float64)


def boundary_values():
    """Near powers of ten and the rounding carries 9.999995 -> 10."""
    out = []
    for e in range(-325, 20):
        for m in (1.0, 9.999995, 9.9999949, 9.9999951, 5.0, 1.0000005, 0.99999949):
            v = m * 10.0 ** e
            if np.isfinite(v) and v != 0:
                out += [v, np.nextafter(v, 0), np.nextafter(v, np.inf)]
    return np.array(out, dtype=np.float64)


def test_format_g6_matches_printf(sid):
    vals = np.concatenate([sample_doubles(100_000, seed=3), tie_values(), boundary_values()])
    bad = []
    ties = 0
    for v in vals:
        v = float(v)
        want = printf_g(v)
        if abs(v) >= 2.0 ** 63 and np.isfinite(v):
            continue   # outside the device formatter's range by design
        got = sid.format_g6(v)
        if got != want:
            bad.append((v, got, want))
            if len(bad) > 5:
                break
    assert not bad, bad
    assert len(tie_values()) > 100


def test_format_g6_range_error(sid):
    import pytest
    with pytest.raises(sid.SidError) as e:
        sid.format_g6(1e300)
    assert e.value.status == 11
    assert sid.format_g6(2.0 ** 62) == printf_g(2.0 ** 62)


def test_format_g6_fast_path_bulk(sid):
    """The double-arithmetic fast path (fmt.h sid_dec6_fast) on 400k values of
    the confidences' range (p-values down to 1e-300, and 6-digit mantissas
    around each 7th-digit half), against printf."""
    rng = np.random.default_rng(11)
    a = np.exp(-rng.random(200_000) * 690.0)
    d = rng.integers(100_000, 1_000_000, size=200_000)
    e = rng.integers(-300, 12, size=200_000)
    half = (d + 0.5) * 10.0 ** (e.astype(np.float64) - 5)
    b = half * (1.0 + rng.integers(-8, 9, size=200_000) * 2.0 ** -52)
    bad = []
    for v in np.concatenate([a, b]):
        v = float(v)
        if not (0 < v < 2.0 ** 63):
            continue
        got, want = sid.format_g6(v), printf_g(v)
        if got != want:
            bad.append((v, got, want))
            if len(bad) > 5:
                break
    assert not bad, bad
