"""compoundLikelihood on the GPU against the oracle at many (pi, eps)
points over high-coverage profile sets: the points that differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import sid_amd as sid  # noqa: E402
import sid_amd.gpu as G  # noqa: E402
import oracle as O  # noqa: E402
from test_lynch_gpu import high_coverage_counts  # noqa: E402

counts = high_coverage_counts(22, 40_000)
ctx = sid.Context(0, method="likelihood_ratio")
d = G.to_device(counts)
ctx.profile_reset(None)
ctx.profile_accumulate(d.data_ptr(), len(counts), None)
ctx.lynch_setup()
rng = np.random.default_rng(0)
pts = [(1e-3, 1e-3), (1.1e-3, 1e-3), (1e-3, 1.1e-3)] + [(float(a), float(b)) for a, b in
       zip(10 ** rng.uniform(-5, -0.5, 400), 10 ** rng.uniform(-5, -0.3, 400))]
bad = 0
for pi, eps in pts:
    g = ctx.lynch_objective(pi, eps)
    r = O.compound_likelihood(counts, pi, eps)
    if not (g == r or (np.isfinite(r) and abs(g - r) <= 1e-13 * abs(r))):
        bad += 1
        if bad <= 25:
            print(f"pi {pi:.6g} eps {eps:.6g} gpu {g!r} oracle {r!r}", flush=True)
print("bad", bad, "of", len(pts))
code, hom, het, est = G.run_method(counts, "likelihood_ratio", estimate_prior=True)
rc, rcode, rhom, rhet, rest, u = O.call_method(counts, "likelihood_ratio", estimate_prior=True)
print("est", est.heterozygosity, est.error_rate, est.iterations, "oracle", rest.heterozygosity, rest.error_rate,
      rest.iterations)
