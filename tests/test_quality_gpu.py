"""-m quality (call.cpp:291-372) on the device text path
against the oracle restatement (oracle_quality_site: long double, glibc
pow/log, the reference's base/quality index alignment): labels/gt bit-exact,
confidences within 1e-10."""

import numpy as np
import pytest

from helpers import assert_parity
from test_parser import blank, fuzz_lines

pytestmark = pytest.mark.gpu


def gpu_quality(gpu, sid, text, **opts):
    import torch
    ctx = sid.Context(0, method="quality", **opts)
    t = sid.DText(ctx, text)
    n = len(t)
    _, code, hom, het = gpu.device_buffers(n)
    sid.check(sid.lib().sid_call_quality(ctx.h, t.h, code.data_ptr(), hom.data_ptr(), het.data_ptr(), None),
              "quality")
    torch.cuda.synchronize()
    return code[:n].cpu().numpy(), hom[:n].cpu().numpy(), het[:n].cpu().numpy()


@pytest.mark.parametrize("depth,n,seed", [(30.0, 100_000, 3), (200.0, 10_000, 5), (8.0, 50_000, 7)])
@pytest.mark.parametrize("opts", [dict(), dict(snp_prior=0.001), dict(significance_level=0.2),
                                  dict(snp_prior=0.5)], ids=lambda o: str(o))
def test_quality_synthetic(gpu, sid, oracle, depth, n, seed, opts):
    text = sid.synth_text(seed, n, depth, sites_per_chrom=n // 2 + 1, mapq=True)
    code, hom, het = gpu_quality(gpu, sid, text, **opts)
    rc, rcode, rhom, rhet = oracle.call_quality(text, snp_prior=opts.get("snp_prior", -1.0),
                                                significance_level=opts.get("significance_level", 0.05))
    assert rc == 0
    assert_parity(code, hom, het, rcode, rhom, rhet, what=f"quality {opts} {depth}x")
    if depth == 30.0 and not opts:
        assert (code & 0x80).sum() > 10   # het calls happen


def quality_fuzz_lines(seed, n):
    """Fuzzed bases (indels, carets, '.'/',' with odd references) with base and
    mapping quality fields of other lengths (shorter: the reference's undefined
    read past the vector, quality 1 here and in the oracle), high bytes, CR."""
    rng = np.random.default_rng(seed)
    base = [l for l in fuzz_lines(seed, n) if l and not blank(l) and b"\x00" not in l]
    out = []
    qchars = list(b"!\"#5?I]~") + [0x80, 0xE9, 0xFF, 0x0D]
    for l in base:
        f = l.split()
        if len(f) < 5:
            continue
        nb = max(0, len(f[4]) + int(rng.integers(-3, 4)))
        bq = rng.choice(qchars, size=nb).astype(np.uint8).tobytes() if nb else b"I"
        mq = rng.choice(qchars, size=max(0, nb + int(rng.integers(-2, 3)))).astype(np.uint8).tobytes() or b"5"
        out.append(b"\t".join(f[:5] + [bq, mq]))
    return out


@pytest.mark.parametrize("seed", [21, 22])
def test_quality_fuzz(gpu, sid, oracle, seed):
    lines = [l for l in quality_fuzz_lines(seed, 60000) if oracle.call_quality(l + b"\n")[0] == 0]
    text = b"\n".join(lines) + b"\n"
    code, hom, het = gpu_quality(gpu, sid, text)
    rc, rcode, rhom, rhet = oracle.call_quality(text)
    assert rc == 0 and len(code) == len(rcode) > 1000
    assert_parity(code, hom, het, rcode, rhom, rhet, what="quality fuzz")


def test_quality_parse_errors(gpu, sid, oracle):
    ctx = sid.Context(0, method="quality")
    good = b"c1\t1\tA\t3\t.,.\tIII\t555\n"
    cases = {
        good + b"c1\t2\tA\t3\t.,.\tIII\n" + good: 5,                       # missing mapping qualities
        good + b"c1\t2\tA\t3\t.,.\n" + good: 12,                           # no base qualities: SIGSEGV
        good + b"c1\t2\tAC\t3\t.,.\tIII\t555\nc1\t3\tA\t1\t.\n": 4,        # malformed first
        good + b" \t\n" + b"c1\t2\tA\t3\t.,.\tIII\n": 6,                   # blank line first
    }
    for text, status in cases.items():
        with pytest.raises(sid.SidError) as e:
            sid.DText(ctx, text)
        assert e.value.status == status, text
        want = {5: 2, 12: 4, 4: 1, 6: 3}[status]
        assert oracle.call_quality(text)[0] == want
    # the same lines are fine for the other methods
    assert len(sid.DText(sid.Context(0), good + b"c1\t2\tA\t3\t.,.\n")) == 2


@pytest.mark.parametrize("flags", [["-m", "quality"], ["-R", "-m", "quality"], ["-r", "0.01", "-m", "quality"],
                                   ["-p", "0.3", "-m", "quality", "--devices", "3"]], ids=" ".join)
def test_cli_quality_matches_oracle(sid, oracle, tmp_path, flags):
    import subprocess
    p = tmp_path / "q.plp"
    p.write_bytes(sid.synth_text(31, 30_000, 30.0, sites_per_chrom=10_000, mapq=True))
    a = subprocess.run([sid.CLI_PATH] + flags + [str(p)], capture_output=True, timeout=600)
    b = oracle.run_cli([f for f in flags if f not in ("--devices", "3")] + [str(p)])
    assert a.returncode == b.returncode == 0, a.stderr
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr


def test_cli_quality_errors_match_oracle(sid, oracle, tmp_path):
    import subprocess
    good = b"c1\t1\tA\t3\t.,.\tIII\t555\n"
    for tag, text in {"nomq": good * 3 + b"c1\t2\tA\t3\t.,.\tIII\n",
                      "nobq": good + b"c1\t2\tA\t3\t.,.\n" + b"c1\t2\tAC\t3\t.,.\n",
                      "six_cols": b"c1\t1\tA\t3\t.,.\tIII\n"}.items():
        p = tmp_path / f"{tag}.plp"
        p.write_bytes(text)
        a = subprocess.run([sid.CLI_PATH, "-m", "quality", str(p)], capture_output=True, timeout=600)
        b = oracle.run_cli(["-m", "quality", str(p)])
        assert a.returncode == b.returncode, tag
        assert a.stdout == b.stdout == b"", tag
        assert a.stderr == b.stderr, tag
