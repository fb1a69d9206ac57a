"""-m local parity: HIP kernel (sid_call_local through the C ABI) against the
CPU oracle (call.cpp:213-289 restated in long double).  label/gt bit-exact,
confidences within 1e-10 relative (tests/helpers.py)."""
import numpy as np
import pytest

from helpers import all_profiles, assert_parity

pytestmark = pytest.mark.gpu

OPTION_SETS = [
    dict(),
    dict(site_error_threshold=0.05, significance_level=0.01, snp_prior=1e-3),
    dict(site_error_threshold=0.0),
    dict(site_error_threshold=0.5, snp_prior=0.001),
    dict(snp_prior=1.0),
    dict(snp_prior=2.0),                       # negative prior factor: signed emulation
    dict(site_error_threshold=-0.1),           # negative bases: signed emulation
    dict(site_error_threshold=1e-300),         # underflow to 0 with few errors
    dict(site_error_threshold=2.0),            # never capped
    dict(significance_level=2.0),              # het decided by l2 > l1 alone
    dict(site_error_threshold=float("nan"), significance_level=float("nan"), snp_prior=float("nan")),
    dict(site_error_threshold=float("inf")),
]


def oracle_opts(o):
    return dict(snp_prior=o.get("snp_prior", -1.0), site_error_threshold=o.get("site_error_threshold", 0.1),
                significance_level=o.get("significance_level", 0.05))


def check(gpu, oracle, counts, what, **o):
    got = gpu.run_local(counts, **o)
    ref = oracle.call_local(counts, **oracle_opts(o))
    assert_parity(*got, *ref, what=what)


def test_exhaustive_default_c40(gpu, oracle):
    check(gpu, oracle, all_profiles(40), "all profiles c<=40")


@pytest.mark.parametrize("o", OPTION_SETS, ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()) or "default")
def test_exhaustive_options_c24(gpu, oracle, o):
    check(gpu, oracle, all_profiles(24), f"c<=24 {o}", **o)


@pytest.mark.parametrize("depth,n,seed", [(30.0, 1_000_000, 2), (200.0, 150_000, 5), (3.0, 100_000, 1)])
def test_synthetic(gpu, oracle, sid, depth, n, seed):
    counts = sid.synth_counts_host(seed, n, depth)
    check(gpu, oracle, counts, f"synthetic {depth}x")


def test_deep_and_extreme_counts(gpu, oracle):
    rng = np.random.default_rng(0)
    parts = [
        rng.integers(0, 3000, size=(20000, 4)),                 # c >= 1024: emulated path
        rng.integers(0, 65536, size=(5000, 4)),                 # up to uint16 max
        np.array([[65535, 0, 0, 0], [65535, 65535, 65535, 65535], [16384] * 4, [30000, 30000, 0, 0],
                  [1023, 0, 0, 0], [1024, 0, 0, 0], [1000, 23, 0, 0], [2000, 100, 50, 25],
                  [0, 0, 0, 0], [1, 0, 0, 0], [0, 0, 0, 1], [5, 5, 5, 5]]),
    ]
    deep_hom = np.zeros((4000, 4), np.int64)
    deep_hom[:, 0] = rng.integers(500, 5000, size=4000)
    deep_hom[:, 1] = rng.integers(0, 40, size=4000)
    parts.append(deep_hom)
    counts = np.concatenate(parts).astype(np.uint16)
    for o in [dict(), dict(site_error_threshold=1e-3), dict(snp_prior=0.5), dict(site_error_threshold=0.0)]:
        check(gpu, oracle, counts, f"deep {o}", **o)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 7, 1023, 4097])
def test_ragged_sizes_and_offsets(gpu, oracle, sid, n):
    counts = sid.synth_counts_host(17, n + 1, 30.0)
    check(gpu, oracle, counts[:n], f"n={n}")
    check(gpu, oracle, counts[1:], f"offset n={n}")


def test_unaligned_device_pointers(gpu, oracle, sid):
    import torch
    n = 1001
    counts = sid.synth_counts_host(4, n + 1, 30.0)
    d = gpu.to_device(counts)
    code = torch.empty(n + 3, dtype=torch.uint8, device="cuda")
    hom = torch.empty(n + 1, dtype=torch.float64, device="cuda")
    het = torch.empty(n + 1, dtype=torch.float64, device="cuda")
    ctx = sid.Context(0)
    # counts shifted by one site (8-B aligned only), code by one byte
    ctx.call_local(d.data_ptr() + 8, n, code.data_ptr() + 1, hom.data_ptr() + 8, het.data_ptr() + 8, None)
    torch.cuda.synchronize()
    ref = oracle.call_local(counts[1:])
    assert_parity(code[1:n + 1].cpu().numpy(), hom[1:].cpu().numpy(), het[1:].cpu().numpy(), *ref,
                  what="unaligned")
    with pytest.raises(sid.SidError):   # profile_t must be 8-B aligned
        ctx.call_local(d.data_ptr() + 2, n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), None)
    ctx.close()


def test_empty_input(gpu):
    code, hom, het = gpu.run_local(np.zeros((0, 4), np.uint16))
    assert len(code) == 0


def _table_coverage_profiles():
    """Every (nf, ns, r2) class around the table borders: nf across the LDS
    (256) and second-level (512) limits, ns across 8 and 128, the minor
    counts split over two bases across r2 = 4 and 8, the major in every
    position."""
    rows = []
    for nf in (0, 1, 30, 200, 255, 256, 257, 300, 511, 512, 513, 700, 1023):
        for ns in (0, 1, 7, 8, 9, 63, 64, 100, 127, 128, 129):
            if ns > nf:
                continue
            for r2 in (0, 1, 3, 4, 5, 7, 8, 9, 20):
                a = min(r2, ns)
                b = r2 - a
                if b > ns:
                    continue
                for f in range(4):
                    p = [ns, a, b]
                    p.insert(f, nf)
                    rows.append(p)
    return np.array(rows, np.uint16)


@pytest.mark.parametrize("tail", ["1", "0"])
def test_second_level_table_borders(gpu, oracle, sid, monkeypatch, tail):
    """Sites the LDS class table misses, resolved inline through the
    second-level table (SID_TABLE_TAIL=1, the default) or all by the fix-up
    kernel (0): the same outputs as the oracle either way, at the borders of
    both tables and mixed into 30x/200x streams."""
    monkeypatch.setenv("SID_TABLE_TAIL", tail)   # read when the context is created
    border = _table_coverage_profiles()
    rng = np.random.default_rng(17)
    counts = np.concatenate([sid.synth_counts_host(5, 60_000, 200.0), border,
                             sid.synth_counts_host(2, 60_000, 30.0)])
    counts = counts[rng.permutation(len(counts))]
    check(gpu, oracle, counts, f"table borders tail={tail}")
    check(gpu, oracle, border, f"table borders only tail={tail}", snp_prior=1e-3, site_error_threshold=0.05)
