"""Product host parser (sid_parse_text, parse.cpp) against the REFERENCE's own
pileup.cpp (oracle/_ref) and the oracle restatement, on synthetic and fuzzed
pileup text.  CPU only."""
import numpy as np
import pytest

ALPH = b".,ACGTacgtNn*$^+-0123456789<>#]!"


def fuzz_lines(seed, n):
    rng = np.random.default_rng(seed)
    seps = [b" ", b"\t", b"  ", b"\t\t", b" \t"]
    refs = [b"A", b"c", b"G", b"t", b"N", b"n", b"^", b"+", b"-", b".", b",", b"*", b"AC", b"\xe9"]
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.03:
            out.append(b"")
            continue
        ntok = int(rng.choice([1, 2, 3, 4, 5, 5, 5, 6, 6, 6, 7]))
        toks = [b"chr" + str(int(rng.integers(0, 30))).encode() if rng.random() < 0.9 else b"x\rY",
                str(int(rng.integers(-5, 10**int(rng.integers(1, 19)))) * int(rng.choice([1, 1, 1, 1000]))).encode()
                if rng.random() < 0.9 else bytes(rng.choice([b"+7", b"\x0b12", b"abc", b"-0", b"99999999999999999999"])),
                refs[int(rng.integers(0, len(refs)))],
                str(int(rng.integers(0, 100))).encode(),
                bytes(rng.choice(list(ALPH), size=int(rng.integers(1, 60)))) if rng.random() < 0.95 else b"*",
                b"IIIII",
                b"]]]"]
        line = toks[0]
        for t in toks[1:ntok]:
            line += seps[int(rng.integers(0, len(seps)))] + t
        if rng.random() < 0.1:
            line = seps[int(rng.integers(0, len(seps)))] + line
        if rng.random() < 0.05:
            line += b"\r"
        if rng.random() < 0.02:
            k = int(rng.integers(0, len(line)))
            line = line[:k] + b"\x00" + line[k:]
        if rng.random() < 0.02:
            line = b" \t"
        out.append(line)
    return out


def product_line(sid, line):
    try:
        s = sid.parse_text(line + b"\n")
    except sid.SidError as e:
        return ("ERR", {4: "std::invalid_argument", 6: "std::logic_error"}[e.status])
    if len(s) == 0:
        return None
    name = s.chroms[0][1].decode("latin-1")
    return ("OK", name, int(s.positions[0])) + tuple(int(x) for x in s.counts[0])


def blank(line):
    # only separators before the end of the C string: the reference assigns a
    # NULL char* to std::string (pileup.cpp:18) and dies with SIGSEGV
    return line.split(b"\x00")[0].strip(b" \t") == b"" and line != b""


def ref_lines(oracle, lines):
    lines = [l for l in lines if not blank(l)]
    text = b"\n".join(lines) + b"\n"
    out = oracle.ref_pileup("lines", text).split(b"\n")[:-1]
    res = []
    for o in out:
        f = o.split(b"\t")
        if f[0] == b"OK":
            res.append(("OK", f[1].decode("latin-1"), int(f[2])) + tuple(int(x) for x in f[3:7]))
        else:
            res.append(("ERR", f[1].decode()))
    return res


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_against_reference_pileup_cpp(sid, oracle, seed):
    if not oracle.ref_pileup_available():
        pytest.skip("oracle/_ref not built")
    lines = fuzz_lines(seed, 1500)
    ref = ref_lines(oracle, lines)
    for l in lines:
        if blank(l):
            assert product_line(sid, l) == ("ERR", "std::logic_error")
    lines = [l for l in lines if not blank(l)]
    mine = [product_line(sid, l) for l in lines]
    mine = [m for m in mine if m is not None]
    assert len(mine) == len(ref)
    for a, b, l in zip(mine, ref, [l for l in lines if l]):
        assert a == b, l


def test_blank_line_crashes_reference(sid, oracle):
    import subprocess
    if not oracle.ref_pileup_available():
        pytest.skip("oracle/_ref not built")
    for l in (b" \t", b"\t", b"  ", b"\x00abc", b" \x00x"):
        r = subprocess.run([oracle.REF_PILEUP, "lines"], input=l + b"\n", capture_output=True)
        assert r.returncode == -11, l          # SIGSEGV inside std::string::assign(nullptr)
        with pytest.raises(sid.SidError) as e:
            sid.parse_text(l + b"\n")
        assert e.value.status == 6


def test_synthetic_against_reference_pileup_cpp(sid, oracle):
    if not oracle.ref_pileup_available():
        pytest.skip("oracle/_ref not built")
    text = sid.synth_text(11, 3000, 30.0, sites_per_chrom=1000)
    ref = ref_lines(oracle, text.split(b"\n")[:-1])
    s = sid.parse_text(text)
    assert len(ref) == len(s) == 3000
    for i, r in enumerate(ref):
        name = [nm for st, nm in s.chroms if st <= i][-1].decode()
        assert r == ("OK", name, int(s.positions[i])) + tuple(int(x) for x in s.counts[i])


@pytest.mark.parametrize("depth,seed", [(30.0, 1), (200.0, 5), (0.5, 9)])
def test_synth_text_parses_to_synth_counts(sid, depth, seed):
    n = 20000 if depth < 100 else 4000
    text = sid.synth_text(seed, n, depth, first=12345, sites_per_chrom=7000)
    s = sid.parse_text(text)
    assert len(s) == n
    assert np.array_equal(s.counts, sid.synth_counts_host(seed, n, depth, first=12345))
    # positions / chromosome runs of the sharded generator
    g = 12345 + np.arange(n)
    assert np.array_equal(s.positions, (g % 7000 + 1).astype(np.int32))
    assert [int(name[3:]) for _, name in s.chroms] == sorted(set((g // 7000 + 1).tolist()))


def test_threads_do_not_change_the_result(sid):
    text = sid.synth_text(3, 60000, 30.0, sites_per_chrom=9999)
    base = sid.parse_text(text, threads=1)
    for t in (2, 3, 8, 16):
        s = sid.parse_text(text, threads=t)
        assert np.array_equal(s.counts, base.counts) and np.array_equal(s.positions, base.positions)
        assert s.chroms == base.chroms


def test_first_error_line_and_kind(sid):
    good = sid.synth_text(1, 1000, 30.0)
    lines = good.split(b"\n")
    bad = b"\n".join(lines[:700] + [b"chr1\t5\tAC\t3\t...\tIII"] + lines[700:820] + [b"\t"] + lines[820:])
    with pytest.raises(sid.SidError) as e:
        sid.parse_text(bad, threads=8)
    assert e.value.status == 4 and e.value.line == 700
    bad2 = b"\n".join(lines[:10] + [b" \t "] + lines[10:])
    with pytest.raises(sid.SidError) as e:
        sid.parse_text(bad2, threads=4)
    assert e.value.status == 6 and e.value.line == 10


def test_edge_semantics(sid):
    # uint16 wrap (pileup.hpp:7) and indel/caret skipping
    s = sid.parse_text(b"c\t1\tA\t0\t" + b"." * 65537 + b"\t*\n")
    assert s.counts[0].tolist() == [1, 0, 0, 0]
    s = sid.parse_text(b"c\t1\tA\t0\t+99999999999999999999999A.\t*\n")
    assert s.counts[0].tolist() == [0, 0, 0, 0]
    s = sid.parse_text(b"c\t-12\t+\t0\t..+2AA,\t*\n")   # '.' acts as '+' when ref is '+'
    assert s.counts[0].tolist() == [0, 0, 0, 0] and s.positions[0] == -12
    s = sid.parse_text(b"c 99999999999 a 0 .,\n")       # atoi = (int)strtol
    assert s.positions[0] == np.int32(np.int64(99999999999).astype(np.int32))
    assert s.counts[0].tolist() == [2, 0, 0, 0]
    assert len(sid.parse_text(b"")) == 0 and len(sid.parse_text(b"\n\n\n")) == 0


def test_fuzz_against_committed_reference_vectors(sid):
    """Same corpus as above, against the reference's outputs committed in
    tests/golden/ref_pileup_fuzz.tsv.gz (works where /root/reference is absent)."""
    import gzip
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_pileup_fuzz.tsv.gz")
    ref = []
    for o in gzip.open(path).read().split(b"\n")[:-1]:
        f = o.split(b"\t")
        if f[0] == b"OK":
            ref.append(("OK", f[1].decode("latin-1"), int(f[2])) + tuple(int(x) for x in f[3:7]))
        else:
            ref.append(("ERR", f[1].decode()))
    lines = [l for s in (1, 2, 3) for l in fuzz_lines(s, 1500) if l and not blank(l)]
    mine = [product_line(sid, l) for l in lines]
    assert mine == ref
