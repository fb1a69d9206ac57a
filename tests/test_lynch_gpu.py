"""Lynch ML path parity: device histogram, GPU
objective + host Nelder-Mead, per-profile classification and per-site lookup
against the oracle (lynch.cpp/optimization.hpp/stats.cpp/call.cpp restated,
long double).  (pi-hat, eps-hat) must come out bit-identical (same simplex
trajectory), labels/gt bit-exact, confidences within 1e-10."""
import numpy as np
import pytest

from helpers import assert_parity

pytestmark = pytest.mark.gpu


def table_via_gpu(gpu, sid, counts, chunks=1):
    import torch
    ctx = sid.Context(0, method="likelihood_ratio")
    d = gpu.to_device(counts)
    ctx.profile_reset(None)
    n = len(counts)
    bounds = np.linspace(0, n, chunks + 1).astype(int)
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        ctx.profile_accumulate(d.data_ptr() + 8 * int(lo), int(hi - lo), None)
    torch.cuda.synchronize()
    k, c = ctx.profile_table()
    ctx.close()
    return k, c


@pytest.mark.parametrize("chunks", [1, 3])
def test_histogram_matches_countUniqueProfiles(gpu, sid, oracle, chunks):
    counts = sid.synth_counts_host(3, 300_000, 30.0)
    k, c = table_via_gpu(gpu, sid, counts, chunks)
    rows, _, u = oracle.unique_profiles(counts)
    assert len(k) == u
    assert k.tolist() == [int(sid.profile_key(np.array([p], np.uint16))[0]) for p, _, _ in rows]
    assert c.tolist() == [cnt for _, cnt, _ in rows]


def test_histogram_many_distinct_grows_table(gpu, sid, oracle):
    rng = np.random.default_rng(1)
    counts = rng.integers(0, 200, size=(400_000, 4)).astype(np.uint16)   # ~all distinct
    counts[::5] = counts[1]
    counts[7] = [65535, 65535, 65535, 65535]                              # sentinel-valued key
    k, c = table_via_gpu(gpu, sid, counts, chunks=2)
    kk, cc = np.unique(sid.profile_key(counts), return_counts=True)
    assert k.tolist() == kk.tolist() and c.tolist() == cc.tolist()


def test_objective_matches_compoundLikelihood(gpu, sid, oracle):
    counts = sid.synth_counts_host(3, 200_000, 30.0)
    ctx = sid.Context(0, method="likelihood_ratio")
    d = gpu.to_device(counts)
    ctx.profile_reset(None)
    ctx.profile_accumulate(d.data_ptr(), len(counts), None)
    est = ctx.lynch_setup()
    assert np.allclose(list(est.dist), oracle.distribution(counts), rtol=0, atol=0)
    worst = 0.0
    for pi, eps in [(1e-3, 1e-3), (1.1e-3, 1e-3), (1e-3, 1.1e-3), (5e-4, 8e-3), (0.2, 0.05),
                    (0.0, 0.01), (1e-3, 0.0), (1.0, 0.5), (-1e-9, 0.1), (0.5, 1.5)]:
        g = ctx.lynch_objective(pi, eps)
        r = oracle.compound_likelihood(counts, pi, eps)
        if r == g:
            continue
        rel = abs(g - r) / abs(r)
        worst = max(worst, rel)
        assert rel < 1e-13, (pi, eps, g, r)
    ctx.close()


CASES = [
    ("likelihood_ratio", dict(estimate_prior=True)),
    ("likelihood_ratio", dict()),
    ("likelihood_ratio", dict(significance_level=0.2)),
    ("bayes", dict()),
    ("local", dict(estimate_prior=True)),
]


@pytest.mark.parametrize("depth,n,seed", [(30.0, 100_000, 3), (200.0, 20_000, 5), (8.0, 50_000, 7)])
@pytest.mark.parametrize("method,o", CASES, ids=lambda x: str(x))
def test_method_parity(gpu, sid, oracle, depth, n, seed, method, o):
    counts = sid.synth_counts_host(seed, n, depth)
    code, hom, het, est = gpu.run_method(counts, method, **o)
    rc, rcode, rhom, rhet, rest, u = oracle.call_method(counts, method, **o)
    assert rc == 0
    assert (est.heterozygosity, est.error_rate, est.iterations, est.converged) == \
        (rest.heterozygosity, rest.error_rate, rest.iterations, rest.converged)
    if method != "local":
        assert est.n_unique == u
    assert_parity(code, hom, het, rcode, rhom, rhet, what=f"{method} {o} {depth}x")


def test_merged_tables_equal_single_context(gpu, sid, oracle):
    import torch
    counts = sid.synth_counts_host(9, 120_000, 30.0)
    parts = [counts[:50_000], counts[50_000:]]
    tables = [table_via_gpu(gpu, sid, p) for p in parts]
    from sid_amd.dist import merge_profile_tables
    k, c = merge_profile_tables(tables)
    outs = []
    for p in parts:
        ctx = sid.Context(0, method="likelihood_ratio", estimate_prior=True)
        d = gpu.to_device(p)
        ctx.profile_reset(None)
        ctx.profile_accumulate(d.data_ptr(), len(p), None)
        ctx.profile_load(k, c)
        ctx.lynch_prepare()
        _, code, hom, het = gpu.device_buffers(len(p))
        ctx.lookup_sites(d.data_ptr(), len(p), code.data_ptr(), hom.data_ptr(), het.data_ptr(), None)
        torch.cuda.synchronize()
        outs.append((code[:len(p)].cpu().numpy(), hom[:len(p)].cpu().numpy(), het[:len(p)].cpu().numpy()))
        ctx.close()
    code = np.concatenate([o[0] for o in outs])
    hom = np.concatenate([o[1] for o in outs])
    het = np.concatenate([o[2] for o in outs])
    rc, rcode, rhom, rhet, rest, u = oracle.call_method(counts, "likelihood_ratio", estimate_prior=True)
    assert_parity(code, hom, het, rcode, rhom, rhet, what="merged tables")


def test_no_profile_with_coverage_4(gpu, sid):
    counts = np.array([[1, 0, 0, 0], [0, 2, 1, 0], [0, 0, 0, 0]], np.uint16)
    with pytest.raises(sid.SidError) as e:
        gpu.run_method(counts, "likelihood_ratio")
    assert e.value.status == 9
    code, hom, het, est = gpu.run_method(counts, "local", estimate_prior=True)  # -R local still runs
    assert len(code) == 3


def _all_small_profiles():
    """Every profile with counts <= 5, plus the dense-code borders: max count
    63/64 with the others 0..4 in every position (sid_math.h sid_dense_code)."""
    g = np.stack(np.meshgrid(*[np.arange(6)] * 4, indexing="ij"), -1).reshape(-1, 4)
    rows = [g]
    for m in (62, 63, 64, 65):
        o = np.stack(np.meshgrid(*[np.arange(5)] * 3, indexing="ij"), -1).reshape(-1, 3)
        for f in range(4):
            p = np.insert(o, f, m, axis=1)
            rows.append(p)
    return np.concatenate(rows).astype(np.uint16)


def test_histogram_dense_code_borders(gpu, sid):
    base = _all_small_profiles()
    rng = np.random.default_rng(5)
    counts = base[rng.integers(0, len(base), 500_000)]
    counts[:len(base)] = base   # every profile at least once
    for lo, hi in ((0, len(counts)), (1, len(counts)), (1, len(counts) - 2)):   # aligned / unaligned / odd
        k, c = table_via_gpu(gpu, sid, counts[lo:hi])
        kk, cc = np.unique(sid.profile_key(counts[lo:hi]), return_counts=True)
        assert k.tolist() == kk.tolist() and c.tolist() == cc.tolist()


def test_histogram_fallback_list_overflow(gpu, sid, monkeypatch):
    monkeypatch.setenv("SID_HIST_LIST_CAP", "16")   # read at the context's first accumulate
    counts = sid.synth_counts_host(11, 200_000, 30.0)
    counts[100:20_000:7] = [40, 30, 9, 65535]        # non-dense profiles, far more than 16
    k, c = table_via_gpu(gpu, sid, counts, chunks=2)
    kk, cc = np.unique(sid.profile_key(counts), return_counts=True)
    assert k.tolist() == kk.tolist() and c.tolist() == cc.tolist()


def test_context_reuse_and_unaligned_lookup(gpu, sid, oracle):
    """Two full runs on one context (state cleared by profile_reset); the lookup
    through an 8-B-offset counts pointer and an odd site count (scalar tail)."""
    import torch
    counts = sid.synth_counts_host(13, 60_001, 30.0)
    ctx = sid.Context(0, method="likelihood_ratio", estimate_prior=True)
    d = gpu.to_device(np.concatenate([np.zeros((1, 4), np.uint16), counts]))
    d2 = gpu.to_device(counts)
    n = len(counts)
    res = []
    for ptr, off in ((d.data_ptr() + 8, 1), (d2.data_ptr(), 0)):   # unaligned, then aligned + odd tail
        ctx.profile_reset(None)
        ctx.profile_accumulate(ptr, n, None)
        ctx.lynch_prepare()
        _, code, hom, het = gpu.device_buffers(n + 1)
        ctx.lookup_sites(ptr, n, code.data_ptr() + off, hom.data_ptr() + 8 * off, het.data_ptr() + 8 * off, None)
        torch.cuda.synchronize()
        res.append((code[off:n + off].cpu().numpy(), hom[off:n + off].cpu().numpy(),
                    het[off:n + off].cpu().numpy()))
    ctx.close()
    rc, rcode, rhom, rhet, rest, u = oracle.call_method(counts, "likelihood_ratio", estimate_prior=True)
    for code, hom, het in res:
        assert_parity(code, hom, het, rcode, rhom, rhet, what="reuse/unaligned")


@pytest.mark.parametrize("depth,n,seed", [(30.0, 80_000, 3), (200.0, 20_000, 5), (8.0, 50_000, 7)])
def test_prefetch_policy_keeps_trajectory(gpu, sid, oracle, monkeypatch, depth, n, seed):
    """The Nelder-Mead estimate on the device (one cooperative launch,
    SID_NM_DEVICE=1) and driven from the host (0, the default), each with and without the
    next iteration's candidates evaluated ahead (SID_NM_LOOKAHEAD): the same
    (pi, eps), iterations, evaluations and outputs, equal to the oracle's."""
    counts = sid.synth_counts_host(seed, n, depth)
    res = {}
    for dev in ("0", "1"):
        for la in ("0", "1"):
            monkeypatch.setenv("SID_NM_DEVICE", dev)     # read when the profiles are set up
            monkeypatch.setenv("SID_NM_LOOKAHEAD", la)
            res[dev + la] = gpu.run_method(counts, "likelihood_ratio", estimate_prior=True)
    c1, h1, t1, e1 = res["01"]
    for key, (c0, h0, t0, e0) in res.items():
        assert (e0.heterozygosity, e0.error_rate, e0.iterations, e0.evaluations, e0.converged) == \
            (e1.heterozygosity, e1.error_rate, e1.iterations, e1.evaluations, e1.converged), key
        assert np.array_equal(c0, c1) and np.array_equal(h0.view(np.int64), h1.view(np.int64)) \
            and np.array_equal(t0.view(np.int64), t1.view(np.int64)), key
    rc, rcode, rhom, rhet, rest, u = oracle.call_method(counts, "likelihood_ratio", estimate_prior=True)
    assert (e1.heterozygosity, e1.error_rate, e1.iterations) == (rest.heterozygosity, rest.error_rate,
                                                                 rest.iterations)
    assert_parity(c1, h1, t1, rcode, rhom, rhet, what=f"prefetch {depth}x")


@pytest.mark.parametrize("method,o", [("likelihood_ratio", dict(estimate_prior=True)), ("bayes", dict()),
                                      ("local", dict(estimate_prior=True))], ids=lambda x: str(x))
def test_device_estimate_edge_tables(gpu, sid, oracle, monkeypatch, method, o):
    """Small and degenerate profile tables through the device estimate: a
    single profile with one base only (the het mixture is 0/0, every L is
    NaN, the objective is -0.0 everywhere and the simplex runs its 1000
    iterations), one base plus a rare second, a handful of profiles, and a
    table whose slices exceed one block per CU — the same estimate as the
    host driver and the oracle, and the oracle's outputs."""
    rng = np.random.default_rng(17)
    tables = [
        np.array([[10, 0, 0, 0]] * 50, np.uint16),
        np.array([[0, 0, 7, 0]] * 20 + [[0, 0, 9, 1]] * 3, np.uint16),
        np.array([[5, 5, 0, 0], [9, 0, 1, 0], [0, 12, 0, 0], [3, 3, 3, 3], [40, 2, 0, 1]] * 40, np.uint16),
        rng.integers(0, 30, (70_000, 4)).astype(np.uint16),   # U ~ 67k: more slices than blocks
    ]
    for ti, t in enumerate(tables):
        out = {}
        for dev in ("0", "1"):
            monkeypatch.setenv("SID_NM_DEVICE", dev)
            try:
                out[dev] = gpu.run_method(t, method, **o)
            except sid.SidError as e:
                out[dev] = e.status
        if isinstance(out["0"], int):
            assert out["1"] == out["0"]
            continue
        (c0, h0, t0, e0), (c1, h1, t1, e1) = out["0"], out["1"]
        assert (e0.heterozygosity, e0.error_rate, e0.iterations, e0.evaluations) == \
            (e1.heterozygosity, e1.error_rate, e1.iterations, e1.evaluations)
        assert np.array_equal(c0, c1) and np.array_equal(h0.view(np.int64), h1.view(np.int64))
        if ti == len(tables) - 1:
            continue   # the oracle needs ~80 s for 67k profiles; the host driver is pinned to it above
        rc, rcode, rhom, rhet, rest, u = oracle.call_method(t, method, **o)
        assert rc == 0 and (e1.heterozygosity, e1.error_rate, e1.iterations) == \
            (rest.heterozygosity, rest.error_rate, rest.iterations)
        assert_parity(c1, h1, t1, rcode, rhom, rhet, what=f"device estimate edge table {method}")


def high_coverage_counts(seed, n):
    """30x sites plus profiles of coverage 500-17000 whose likelihoods fall
    in the long double's denormal range (a few units of 2^-16445 before M
    multiplies them), underflow, or meet an M over LDBL_MAX (0 * inf)."""
    rng = np.random.default_rng(seed)
    base = np.asarray(__import__("sid_amd").synth_counts_host(seed, n, 30.0)).copy()
    rows = []
    for _ in range(3000):
        c = int(rng.choice([500, 1000, 1500, 2000, 3148, 3150, 5000, 13000]))
        f = rng.dirichlet(rng.choice([[1, 1, 1, 1], [20, 20, 1, 1], [40, 1, 1, 1], [2, 2, 2, 4]]))
        p = rng.multinomial(c, f)
        rows.append(np.minimum(p, 65535))
    for p in ([630, 630, 629, 1259], [630, 630, 1259, 629], [630, 1260, 629, 629], [1260, 630, 629, 629]):
        rows += [p] * 5
    hc = np.asarray(rows, np.uint16)
    out = np.concatenate([base, hc])
    return out[rng.permutation(len(out))]


def test_objective_in_the_long_double_denormal_range(gpu, sid, oracle):
    """compoundLikelihood (lynch.cpp:37-61) where lynch.hpp:57-96's long
    doubles are denormal, zero or infinite: the emulated mixture (every
    operation rounded as the x87 format rounds it) against the oracle's real
    long doubles."""
    counts = high_coverage_counts(21, 50_000)
    ctx = sid.Context(0, method="likelihood_ratio")
    d = gpu.to_device(counts)
    ctx.profile_reset(None)
    ctx.profile_accumulate(d.data_ptr(), len(counts), None)
    ctx.lynch_setup()
    for pi, eps in [(1e-3, 1e-3), (1.1e-3, 1e-3), (1e-3, 1.1e-3), (5e-4, 8e-3), (0.2, 0.05), (1e-3, 1e-2),
                    (1e-3, 3e-4), (0.0, 1e-3), (1.0, 1e-3)]:
        g = ctx.lynch_objective(pi, eps)
        r = oracle.compound_likelihood(counts, pi, eps)
        assert g == r or abs(g - r) <= 1e-13 * abs(r), (pi, eps, g, r)
    ctx.close()


@pytest.mark.parametrize("method,o", CASES[:2] + CASES[3:], ids=lambda x: str(x))
def test_method_parity_high_coverage(gpu, sid, oracle, method, o):
    counts = high_coverage_counts(22, 40_000)
    code, hom, het, est = gpu.run_method(counts, method, **o)
    rc, rcode, rhom, rhet, rest, u = oracle.call_method(counts, method, **o)
    assert rc == 0
    assert (est.heterozygosity, est.error_rate, est.iterations, est.converged) == \
        (rest.heterozygosity, rest.error_rate, rest.iterations, rest.converged)
    assert_parity(code, hom, het, rcode, rhom, rhet, what=f"{method} {o} high coverage")
