"""Pin the CPU oracle (and the product's host parser) to the reference's own
known answers: the Catch KATs of test/*.cpp (tests/golden/kat.json) and, when
oracle/_ref is built, the reference's pileup.cpp itself.  CPU only."""
import json
import math
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat.json")))


def line_for(bases, ref):
    # a minimal pileup line whose read-bases field is `bases`
    return b"c\t1\t" + ref.encode() + b"\t0\t" + (bases.encode() if bases else b"*") + b"\t*"


@pytest.mark.parametrize("k", KAT["read_bases"], ids=lambda k: k["cite"])
def test_read_bases_oracle(oracle, k):
    assert oracle.read_bases(k["bases"].encode(), k["ref"].encode()).tolist() == k["counts"]


@pytest.mark.parametrize("k", KAT["read_bases"], ids=lambda k: k["cite"])
def test_read_bases_product(sid, k):
    if k["bases"] == "":
        pytest.skip("an empty read-bases field is not representable inside a tab-separated line")
    s = sid.parse_text(line_for(k["bases"], k["ref"]))
    assert s.counts[0].tolist() == k["counts"]


@pytest.mark.parametrize("k", KAT["read_bases"], ids=lambda k: k["cite"])
def test_read_bases_reference_build(oracle, k):
    if not oracle.ref_pileup_available():
        pytest.skip("oracle/_ref not built (reference sources absent)")
    if k["bases"] == "":
        pytest.skip("empty field")
    out = oracle.ref_pileup("lines", line_for(k["bases"], k["ref"]) + b"\n").decode().split("\t")
    assert out[0] == "OK" and [int(x) for x in out[3:7]] == k["counts"]


def test_qualities_oracle(oracle):
    import ctypes as C
    for k in KAT["qualities"]:
        buf = (C.c_uint8 * 16)()
        n = oracle.lib().oracle_parse_qualities(k["text"].encode(), buf, 16)
        assert list(buf[:n]) == k["values"], k["cite"]


def test_full_line(oracle, sid):
    k = KAT["line"]
    s = sid.parse_text(k["text"].encode())
    assert s.chroms == [(0, k["chrom"].encode())]
    assert s.positions.tolist() == [k["position"]]
    assert s.counts[0].tolist() == k["counts"]
    if oracle.ref_pileup_available():
        out = oracle.ref_pileup("lines", k["text"].encode() + b"\n").decode().split()
        assert out[:3] == ["OK", k["chrom"], str(k["position"])]
        assert [int(x) for x in out[3:7]] == k["counts"]
        q = oracle.ref_pileup("quals", b"++5D5\nDD55D\n").decode().splitlines()
        assert [int(x) for x in q[0].split()] == k["base_qualities"]
        assert [int(x) for x in q[1].split()] == k["mapping_qualities"]


@pytest.mark.parametrize("k", KAT["unique_profiles"], ids=lambda k: k["cite"])
def test_unique_profiles(oracle, k):
    sites = np.array(k["sites"], np.uint16).reshape(-1, 4)
    rows, _, _ = oracle.unique_profiles(sites)
    assert [[list(p), c] for p, c, _ in rows] == k["unique"]


@pytest.mark.parametrize("k", KAT["distribution"], ids=lambda k: k["cite"])
def test_distribution(oracle, k):
    sites = [p for p, c in k["profiles"] for _ in range(c)]
    d = oracle.distribution(np.array(sites, np.uint16).reshape(-1, 4), min_coverage4=False)
    assert np.allclose(d, k["dist"], rtol=0, atol=1e-15)


def test_distribution_reference_build(oracle):
    if not oracle.ref_pileup_available():
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(7)
    sites = rng.integers(0, 40, size=(5000, 4)).astype(np.uint16)
    sites[::7] = sites[3]  # repeats
    data = "\n".join(" ".join(map(str, r)) for r in sites).encode() + b"\n"
    ref = oracle.ref_pileup("profiles", data).decode().splitlines()
    rows, ptr, u = oracle.unique_profiles(sites)
    assert len(ref) == u + 1
    for line, (p, c, cov) in zip(ref[:-1], rows):
        assert [int(x) for x in line.split()] == list(p) + [c, cov]
    dref = [float(x) for x in ref[-1].split()[1:]]
    d = oracle.distribution(sites, min_coverage4=False)
    assert d.tolist() == dref   # bit-exact


# ---- GSL restatement: chi-square tail and lnGamma against scipy / mpmath ----
def test_chisq_Q_against_scipy_mpmath(oracle):
    import mpmath as mp
    import scipy.special as sp
    mp.mp.dps = 50
    xs = np.concatenate([np.geomspace(1e-12, 1e3, 400), np.linspace(1000, 1400, 50)])
    for x in xs:
        q = oracle.chisq_Q(x)
        t = float(mp.erfc(mp.sqrt(mp.mpf(float(x)) / 2)))
        assert abs(q - t) <= 1e-12 * t, (x, q, t)      # GSL's own accuracy: ~5e-14
        s = sp.chdtrc(1, x)
        assert abs(q - s) <= 1e-12 * s
    assert oracle.chisq_Q(0.0) == 1.0 and oracle.chisq_Q(-1.0) == 1.0
    assert oracle.chisq_Q(1.7976931348623157e308) == 0.0
    assert math.isnan(oracle.chisq_Q(float("nan")))


def test_lngamma_against_scipy(oracle):
    import scipy.special as sp
    for x in [1.5, 3, 4, 10, 31, 100, 1000, 12345, 262141]:
        assert abs(oracle.lngamma(x) - sp.gammaln(x)) <= 1e-13 * max(1, abs(sp.gammaln(x)))
    assert oracle.lngamma(1.0) == 0.0 and oracle.lngamma(2.0) == 0.0


def catch_approx(got, want):
    """Catch v1.9.4's default `== Approx(want)` (test/catch.hpp:2766-2806):
    |got - want| < 100 FLT_EPSILON (1 + max(|got|, |want|))."""
    eps = float(np.finfo(np.float32).eps) * 100
    return abs(got - want) < eps * (1.0 + max(abs(got), abs(want)))


@pytest.mark.parametrize("k", KAT["binomial_pmf"], ids=lambda k: f"n{k['n']}k{k['k']}")
def test_lngamma_binomial_pmf_reference_vectors(oracle, k):
    """The reference's one held set of lnGamma-dependent numbers: 30 binomial
    pmf values (scipy-computed, test/test-likelihoods.cpp:22-49), rebuilt from
    the oracle's restated gsl_sf_lngamma as -m quality's log-binomial does
    (call.cpp:344-349: lnG(n+1) - lnG(n-k+1) - lnG(k+1)), where lnG does not
    cancel.  Checked at Catch's default Approx, and tighter (1e-9 relative)
    wherever the expected value is a normal double."""
    n, kk, p, want = k["n"], k["k"], k["p"], k["pmf"]
    lb = oracle.lngamma(n + 1) - oracle.lngamma(n - kk + 1) - oracle.lngamma(kk + 1)
    got = math.exp(lb + kk * math.log(p) + (n - kk) * math.log(1 - p))
    assert catch_approx(got, want), (got, want)
    if want > 1e-300:
        assert abs(got - want) <= 1e-9 * want, (got, want)
    else:   # the pmf underflows a double (exponent below -745)
        assert got == 0.0 and lb + kk * math.log(p) + (n - kk) * math.log(1 - p) < -745


# ---- outputs the survey observed from the reference build ----
EDGE = (b"c1\t1\tA\t0\t*\t*\n"
        b"c1\t2\tA\t4\tAACC\tIIII\n"
        b"c1\t3\tA\t4\tCCAA\tIIII\n"
        b"c1\t4\tN\t6\t..,,GG\tIIIIII\n"
        b"c1\t5\tA\t4\t.*,N,\tIIII\n"
        b"\n"
        b"c1\t6\tA\t4\t.+2AC,-1T.\tIIII\n"
        b"c1\t7\tG\t12\tGGGGGGCCCCCC\tIIIIIIIIIIII\n"
        b"c1\t8\tC\t41\t" + b"C" * 41 + b"\tIIII\n"
        b"c1\t9\tA\t3\t^I.$.a\tIII\n")


def test_survey_observed_outputs(oracle, tmp_path):
    p = tmp_path / "edge.plp"
    p.write_bytes(EDGE)
    out = oracle.run_cli([str(p)]).stdout.decode().splitlines()
    want = {"1": "hom,TT,1,1", "2": "het,CA,1,0.00358864", "3": "het,CA,1,0.00358864",
            "4": "hom,GG,0.095891,1", "5": "hom,AA,0.0414167,1", "6": "hom,AA,0.0414167,1",
            "7": "het,GC,1,4.5561e-07", "8": "hom,CC,4.73216e-14,1", "9": "hom,AA,0.0414167,1"}
    assert out[0] == "chrom,pos,label,gt,hom_conf,het_conf,conf_type"
    got = {l.split(",")[1]: ",".join(l.split(",")[2:6]) for l in out[1:]}
    assert got == want


def test_bases_vector_kat(oracle):
    # test/test-pileup_parser.cpp:23-35: parseReadBases("AgACgt", 'N').bases
    assert oracle.read_bases_seq(b"AgACgt", b"N") == b"AGACGT"
    # '.'/',' map to the reference; '^' skips the mapping quality; indels skip
    assert oracle.read_bases_seq(b".,^]A$+2CCg-1at", b"c") == b"CCAGT"


def test_quality_line_fields_kat(oracle):
    # test/test-pileup_parser.cpp:37-56: the 7-field line parses (quality mode)
    text = b"chr19\t1337\tA\t6\tAgACgt\t++5D5\tDD55D\n"
    rc, code, hom, het = oracle.call_quality(text)
    assert rc == 0 and len(code) == 1
    # 6 fields: missing mapping qualities; 5 fields: the reference dereferences NULL
    assert oracle.call_quality(b"chr19\t1337\tA\t6\tAgACgt\t++5D5\n")[0] == 2
    assert oracle.call_quality(b"chr19\t1337\tA\t6\tAgACgt\n")[0] == 4
    assert oracle.call_quality(b"chr19\t1337\tAC\t6\tAgACgt\t++5D5\n")[0] == 1


def test_quality_site_by_hand(oracle):
    """call.cpp:311-369 for one site, recomputed with numpy long double."""
    import numpy as np
    from scipy.special import chdtrc
    text = b"c1\t5\tA\t4\tAAAC\tIIII\t5555\n"   # bq 40, mq 20 -> q = 20, e = 0.01
    rc, code, hom, het = oracle.call_quality(text)
    e = 10 ** (20 / -10.)
    lph = np.longdouble(0)
    lpt = np.longdouble(0)
    for b in b"AAAC":
        lph += np.log(1 - e) if b == ord("A") else np.log(e)
        lpt += np.log(1 - 2. / 3. * e)
    n, k = 4, 1
    lb = oracle.lngamma(5) - oracle.lngamma(4) - oracle.lngamma(2)
    lpt += np.longdouble(lb) - n * np.log(np.longdouble(2))
    # here the het model wins: p_hom = LRT(pp2, pp1) = 1, p_het = Q(2 (lpt - lph))
    assert lpt > lph and hom[0] == 1.0
    p = chdtrc(1, float(2 * (lpt - lph)))
    assert abs(het[0] - p) < 1e-12 * p
    assert code[0] == (0 | (1 << 2) | 0x80) if p < 0.05 else code[0] == 0


@pytest.mark.parametrize("method", ["quality", "local"])
def test_oracle_range_equals_the_slice(sid, oracle, tmp_path, method):
    """The CPU baseline's shard harness (ORACLE_RANGE=OFF:LEN, not a reference
    option) reads only the line-aligned bytes [OFF, OFF+LEN) of the file, for
    -m quality as for the other methods: its output equals the oracle over
    that slice written as a file of its own (round 5's quality branch read to
    EOF and took chrom/pos from byte 0)."""
    import os
    text = sid.synth_text(71, 6000, 30.0, sites_per_chrom=2500, mapq=True)
    a = text.index(b"\n", len(text) // 3) + 1
    b = text.index(b"\n", 2 * len(text) // 3) + 1
    whole = tmp_path / "whole.plp"
    whole.write_bytes(text)
    part = tmp_path / "part.plp"
    part.write_bytes(text[a:b])
    ref = oracle.run_cli(["-m", method, str(part)])
    got = oracle.run_cli(["-m", method, str(whole)], env=dict(os.environ, ORACLE_RANGE=f"{a}:{b - a}"))
    assert ref.returncode == 0 and got.returncode == 0
    assert got.stdout == ref.stdout and got.stderr == ref.stderr
    assert got.stdout.count(b"\n") > 1000


@pytest.mark.parametrize("src", ["golden", "synthetic", "edge"])
def test_reference_sources_local_equals_oracle(sid, oracle, tmp_path, src):
    """oracle/_ref/ref_pileup local -- the CPU baseline's "reference sources"
    leg: the reference's pileup.cpp parse, countUniqueProfiles, a profile map
    and call.hpp's operator<< over iostreams, each unique profile's arithmetic
    from the oracle (GSL is absent) -- prints the oracle CLI's -m local CSV
    byte for byte, whole file and over an ORACLE_RANGE byte range."""
    import os
    if not oracle.ref_pileup_available():
        pytest.skip("oracle/_ref not built (no /root/reference)")
    golden = os.path.join(os.path.dirname(__file__), "golden")
    if src == "synthetic":
        p = tmp_path / "s.plp"
        p.write_bytes(sid.synth_text(73, 30_000, 30.0, sites_per_chrom=12_000))
    else:
        p = os.path.join(golden, "c1_10k.plp" if src == "golden" else "edge.plp")
    text = open(p, "rb").read()
    a = text.index(b"\n", len(text) // 4) + 1
    b = text.index(b"\n", len(text) // 2) + 1
    for env in ({}, {"ORACLE_RANGE": f"{a}:{b - a}"}):
        e = dict(os.environ, **env)
        want = oracle.run_cli([str(p)], env=e)
        got = subprocess.run([oracle.REF_PILEUP, "local", str(p)], capture_output=True, env=e)
        assert want.returncode == 0 and got.returncode == 0
        assert got.stdout == want.stdout, (src, env)


@pytest.mark.parametrize("flags", [["-R", "-m", "likelihood_ratio"], ["-m", "bayes"], ["-R", "-m", "local"]],
                         ids=["lr_R", "bayes", "local_R"])
def test_oracle_given_profile_table(sid, oracle, tmp_path, flags):
    """The harness's ORACLE_PROFILE_TABLE (not a reference option): a process
    that reads part of an input (ORACLE_RANGE) but is given the whole input's
    unique-profile table prints exactly the whole run's records for its part
    -- the Lynch estimate and BH are global (call.cpp:62-143) -- which is how
    bench.py checks each rank's records at N ranks."""
    import os
    n = 40_000
    text = sid.synth_text(74, n, 30.0, sites_per_chrom=10 ** 7)
    counts = sid.synth_counts_host(74, n, 30.0)
    keys, cnt = np.unique(sid.profile_key(counts), return_counts=True)
    table = tmp_path / "table.bin"
    np.stack([keys, cnt.astype(np.uint64)], 1).astype(np.uint64).tofile(table)
    p = tmp_path / "all.plp"
    p.write_bytes(text)
    whole = oracle.run_cli(flags + [str(p)])
    assert whole.returncode == 0
    a = text.index(b"\n", len(text) // 2) + 1
    pos0 = int(text[a:].split(b"\t", 2)[1])
    env = dict(os.environ, ORACLE_RANGE=f"{a}:{len(text) - a}", ORACLE_PROFILE_TABLE=str(table))
    part = oracle.run_cli(flags + [str(p)], env=env)
    assert part.returncode == 0
    rows = whole.stdout.split(b"\n")
    tail = [r for r in rows[1:] if r and int(r.split(b",", 2)[1]) >= pos0]
    assert part.stdout == b"\n".join([rows[0]] + tail) + b"\n"
    assert part.stderr == whole.stderr   # (the same table: the same profile count and estimate)
    # without the table the part's own estimate differs
    own = oracle.run_cli(flags + [str(p)], env=dict(os.environ, ORACLE_RANGE=f"{a}:{len(text) - a}"))
    assert own.stderr != whole.stderr
