"""The engine's parse passes against the oracle CLI (the reference's
pileup.cpp / call.cpp / sid.cpp restated), byte for byte: the fast paths (the
tile parse, the per-line and quad parses) and the general routine they hand
lines to.

The texts aim at the fast paths' edge cases (pileup.cpp:13-153):
'^' + mapping quality at every offset of a 16-B window ('^' at a window's last
byte skips the next window's first), '^' runs, '$', indels, CRLF line ends and
NUL or other control bytes after token 4 (their tile goes to the per-line
pass), headers whose token 4 starts 64 or more bytes in, read-bases tokens of
4095-4097 bytes and longer than a 16 KiB tile, multiple and leading
separators, '.'/',' against lower-case and N refs, empty lines, no final
newline; chunk sizes that cut the text anywhere."""
import os
import subprocess

import numpy as np
import pytest

from test_parser import blank, fuzz_lines

pytestmark = pytest.mark.gpu


def cli(sid, args):
    return subprocess.run([sid.CLI_PATH] + list(args), capture_output=True, timeout=600)


def first_diff(a, b):
    """(offset, a's line there, b's line there) of the first byte where a and
    b differ (pytest's own diff of megabyte outputs takes minutes)."""
    n = min(len(a), len(b))
    x, y = np.frombuffer(a[:n], np.uint8), np.frombuffer(b[:n], np.uint8)
    k = int(np.argmax(x != y)) if n and (x != y).any() else n
    s = a.rfind(b"\n", 0, k) + 1
    return k, a[s:a.find(b"\n", k)][:200], b[s:b.find(b"\n", k)][:200]


def same_as_oracle(sid, oracle, path, flags, extra):
    """The CLI against the oracle CLI: stdout, stderr and exit code."""
    b = oracle.run_cli(flags + [str(path)])
    a = cli(sid, extra + flags + [str(path)])
    assert a.returncode == b.returncode, (a.stderr[-300:], b.stderr[-300:])
    same_out = a.stdout == b.stdout
    assert same_out, (extra, flags, first_diff(a.stdout, b.stdout))
    same_err = a.stderr == b.stderr
    assert same_err, (a.stderr[-400:], b.stderr[-400:])
    return b


def mutate(rng, line):
    """One synthetic 30x line with one of the fast paths' edge cases."""
    chrom, pos, ref, depth, bases, qual = line.split(b"\t")[:6]
    r = int(rng.integers(0, 14))
    if r == 0:      # '^' + a mapping-quality byte at random places, sometimes '^^' (a '^' run)
        for _ in range(int(rng.integers(1, 4))):
            k = int(rng.integers(0, len(bases) + 1))
            bases = bases[:k] + b"^" + bytes([int(rng.choice(list(b"I^$.,A+~")))]) + bases[k:]
    elif r == 1:    # '$' read ends
        k = int(rng.integers(0, len(bases) + 1))
        bases = bases[:k] + b"$" + bases[k:]
    elif r == 2:    # an indel
        k = int(rng.integers(0, len(bases) + 1))
        bases = bases[:k] + (b"+2AC" if rng.random() < 0.5 else b"-1t") + bases[k:]
    elif r == 3:    # CRLF
        qual = qual + b"\r"
    elif r == 4:    # a NUL / control byte in the qualities
        k = int(rng.integers(0, len(qual)))
        qual = qual[:k] + bytes([int(rng.choice([0, 1, 11, 13]))]) + qual[k:]
    elif r == 5:    # token 4 starts 60-70 bytes in
        chrom = (b"scaffold_" + chrom + b"_" + b"y" * 80)[: int(rng.integers(40, 60))]
    elif r == 6:    # read bases of about the accumulator's limit (4096) and past a tile (16 KiB)
        n = int(rng.choice([4090, 4094, 4095, 4096, 4097, 4100, 17000]))
        unit = b"ACGT.,acgt$^I"
        bases = (unit * (n // len(unit) + 1))[:n]
    elif r == 7:    # spaces and separator runs, a leading separator
        sep = [b" ", b"\t\t", b" \t", b"\t"]
        out = b"" if rng.random() < 0.5 else b" "
        toks = [chrom, pos, ref, depth, bases, qual]
        line = out + toks[0]
        for t in toks[1:]:
            line += sep[int(rng.integers(0, len(sep)))] + t
        return line
    elif r == 8:    # lower-case, N and '*' refs
        ref = bytes([int(rng.choice(list(b"acgtNn*")))])
    elif r == 9:    # only the first five tokens
        return b"\t".join([chrom, pos, ref, depth, bases])
    return b"\t".join([chrom, pos, ref, depth, bases, qual])


def stress_text(sid, seed, n, depth=30.0):
    rng = np.random.default_rng(seed)
    lines = sid.synth_text(seed, n, depth, sites_per_chrom=n // 3 + 1).split(b"\n")
    out = []
    for ln in lines:
        if not ln:
            continue
        out.append(mutate(rng, ln) if rng.random() < 0.3 else ln)
        if rng.random() < 0.01:
            out.append(b"")   # an empty line (not a site)
    return b"\n".join(out)    # no final newline


@pytest.mark.parametrize("seed,depth", [(41, 30.0), (42, 30.0), (43, 200.0)])
def test_stress_text_equals_oracle(sid, oracle, tmp_path, seed, depth):
    text = stress_text(sid, seed, 6000 if depth > 100 else 20000, depth)
    p = tmp_path / "stress.plp"
    p.write_bytes(text)
    for extra in (["--chunk-bytes", str(1 << 20)], ["--chunk-bytes", "65537", "--devices", "2"],
                  ["--chunk-bytes", "20000"]):
        same_as_oracle(sid, oracle, p, [], extra)
    same_as_oracle(sid, oracle, p, ["-R", "-m", "likelihood_ratio"], ["--chunk-bytes", "300000"])
    if seed == 41:   # the other Lynch-path methods on the same profiles (NaN p-values, denormal likelihoods)
        same_as_oracle(sid, oracle, p, ["-m", "bayes"], ["--chunk-bytes", "300000"])
        same_as_oracle(sid, oracle, p, ["-R", "-m", "local"], ["--chunk-bytes", "300000", "--devices", "2"])
        same_as_oracle(sid, oracle, p, ["-m", "likelihood_ratio", "-p", "0.2"], ["--chunk-bytes", "1000000"])


@pytest.mark.parametrize("seed", [4, 5, 6, 9])
def test_valid_fuzz_lines_equal_oracle(sid, oracle, tmp_path, seed):
    lines = [l for l in fuzz_lines(seed, 4000) if not blank(l)]
    ok = []
    for l in lines:
        try:
            sid.parse_text(l + b"\n")
            ok.append(l)
        except sid.SidError:
            pass
    text = b"\n".join(ok[:1500]) + b"\n\n\n" + b"\n".join(ok[1500:])
    p = tmp_path / "fuzz.plp"
    p.write_bytes(text)
    for extra in (["--chunk-bytes", str(1 << 20)], ["--chunk-bytes", "4096"], ["--chunk-bytes", "9999"]):
        same_as_oracle(sid, oracle, p, [], extra)


@pytest.mark.parametrize("seed", [7, 8])
def test_fuzz_first_error_equals_oracle(sid, oracle, tmp_path, seed):
    """Texts that stop at a malformed line: stdout empty, the same message and
    exit code as the reference, whichever parse pass meets the line."""
    lines = fuzz_lines(seed, 3000)
    rng = np.random.default_rng(seed)
    for trial in range(6):
        k = int(rng.integers(0, len(lines)))
        p = tmp_path / f"e{trial}.plp"
        p.write_bytes(b"\n".join(lines[:k]) + b"\n")
        same_as_oracle(sid, oracle, p, [], ["--chunk-bytes", str(int(rng.choice([4096, 65536, 1 << 20])))])


def test_caret_at_every_window_offset(sid, oracle, tmp_path):
    """'^X' and '^^X' at each of the 16 offsets of a window, in lines whose
    read bases start at every phase."""
    out = []
    for lead in range(16):
        for off in range(40):
            for mq in (b"I", b"^", b"$", b"."):
                bases = b"..,,AC" * 8
                bases = bases[:off] + b"^" + mq + bases[off:]
                chrom = b"c" * (1 + lead)
                out.append(b"\t".join([chrom, str(100 + off).encode(), b"A", b"50", bases, b"I" * 50]))
    p = tmp_path / "caret.plp"
    p.write_bytes(b"\n".join(out) + b"\n")
    for extra in (["--chunk-bytes", str(1 << 20)], ["--chunk-bytes", "7777"]):
        same_as_oracle(sid, oracle, p, [], extra)


def test_caret_at_every_window_offset_long_lines(sid, oracle, tmp_path):
    """The same '^' placements in 200x-long lines (over 256 B on average: the
    quad parse, textpath.hip sid_parse_quad_kernel): a '^' at a window's last
    byte skips the first byte of the next window, which another lane of the
    quad counts; '^^' across that boundary fails in the right lane."""
    out = []
    for lead in range(16):
        for off in range(0, 96):
            for mq in (b"I", b"^", b"$", b"A"):
                bases = b"..,,AC.,gt" * 36
                bases = bases[:off] + b"^" + mq + bases[off:]
                chrom = b"c" * (1 + lead)
                out.append(b"\t".join([chrom, str(100 + off).encode(), b"A", b"370", bases, b"I" * 370]))
    p = tmp_path / "caret_long.plp"
    p.write_bytes(b"\n".join(out) + b"\n")
    for extra in (["--chunk-bytes", str(1 << 20)], ["--chunk-bytes", "77777", "--devices", "2"]):
        same_as_oracle(sid, oracle, p, [], extra)
