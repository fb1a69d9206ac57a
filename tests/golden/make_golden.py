#!/usr/bin/env python3
"""Regenerate the committed fixtures of tests/golden.

  c1_10k.plp            BASELINE.json configs[0] input: 10,000 sites, 30x,
                        seed 1, chr1 (counter-based generator, sid_amd.synth_text)
  edge.plp              hand-written edge cases
  c1_10k.*.csv.gz       expected CSV from the oracle CLI (reference sid.cpp +
                        call.cpp restated; oracle/_build/sid_oracle)
  ref_pileup_fuzz.tsv.gz  the REFERENCE's pileup.cpp (oracle/_ref) on a fuzzed
                        line corpus, so the parser stays pinned where the
                        reference sources are absent (GPU box)

Run from the repo root after `make`.
"""
import gzip
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.dirname(HERE)]

import oracle  # noqa: E402
import sid_amd  # noqa: E402

EDGE = (b"c1\t1\tA\t0\t*\t*\n"
        b"c1\t2\tA\t4\tAACC\tIIII\n"
        b"c1\t3\tA\t4\tCCAA\tIIII\n"
        b"c1\t4\tN\t6\t..,,GG\tIIIIII\n"
        b"c1\t5\tA\t4\t.*,N,\tIIII\n"
        b"\n"
        b"c1\t6\tA\t4\t.+2AC,-1T.\tIIII\n"
        b"c1\t7\tG\t12\tGGGGGGCCCCCC\tIIIIIIIIIIII\n"
        b"c1\t8\tC\t41\t" + b"C" * 41 + b"\tIIII\n"
        b"c1\t9\tA\t3\t^I.$.a\tIII\n"
        b"c2  10 t 5 ,,,,,a IIIII\n"
        b"c2\t11\tg\t7\t..,,TTt$\tIIIIIII\r\n"
        b"c2\t12\tC\t9\tccccGGGGa\tIIIIIIIII\n"
        b"c2\t13\tA\t30\t" + b"." * 15 + b"T" * 15 + b"\t" + b"I" * 30 + b"\n"
        b"c2\t14\tA\t30\t" + b"." * 29 + b"G" + b"\t" + b"I" * 30 + b"\n"
        b"c3\t1\tT\t6\tAACCGG\tIIIIII\n"
        b"c3\t2\tT\t2\t,.\tII\n"
        b"c3\t3\tT\t1\t.\tI\n"
        b"c3\t99999999999\tT\t3\t...\tIII\n")

CSVS = {"local": [], "lr_R": ["-R", "-m", "likelihood_ratio"], "lr": ["-m", "likelihood_ratio"],
        "bayes": ["-m", "bayes"], "local_R": ["-R", "-m", "local"]}


def write_gz(path, data):
    with open(path, "wb") as raw:
        with gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as f:
            f.write(data)


def main():
    c1 = os.path.join(HERE, "c1_10k.plp")
    with open(c1, "wb") as f:
        f.write(sid_amd.synth_text(1, 10_000, 30.0))
    with open(os.path.join(HERE, "edge.plp"), "wb") as f:
        f.write(EDGE)
    for tag, flags in CSVS.items():
        r = oracle.run_cli(flags + [c1], check=True)
        write_gz(os.path.join(HERE, f"c1_10k.{tag}.csv.gz"), r.stdout)
        with open(os.path.join(HERE, f"c1_10k.{tag}.stderr"), "wb") as f:
            f.write(r.stderr)
    if oracle.ref_pileup_available():
        from test_parser import blank, fuzz_lines
        lines = [l for s in (1, 2, 3) for l in fuzz_lines(s, 1500) if l and not blank(l)]
        out = oracle.ref_pileup("lines", b"\n".join(lines) + b"\n")
        write_gz(os.path.join(HERE, "ref_pileup_fuzz.tsv.gz"), out)


if __name__ == "__main__":
    main()
