"""Where the Lynch estimate on a stress text parts from the oracle: the
nucleotide distribution, compoundLikelihood at fixed points, the estimate,
with and without the high-coverage profiles."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import sid_amd as sid  # noqa: E402
import sid_amd.gpu as G  # noqa: E402
import oracle as O  # noqa: E402
from test_parse_stress_gpu import stress_text  # noqa: E402

text = stress_text(sid, 41, 20000, 30.0)
counts = sid.parse_text(text).counts.copy()
cov = counts.astype(np.int64).sum(1)
print("sites", len(counts), "max cov", cov.max(), "cov>1000", int((cov > 1000).sum()), flush=True)
for name, c in [("all", counts), ("cov<=1000", counts[cov <= 1000]), ("cov<=300", counts[cov <= 300])]:
    ctx = sid.Context(0, method="likelihood_ratio")
    d = G.to_device(np.ascontiguousarray(c))
    ctx.profile_reset(None)
    ctx.profile_accumulate(d.data_ptr(), len(c), None)
    est = ctx.lynch_setup()
    od = O.distribution(c)
    print(name, "dist equal", list(est.dist) == list(od), list(est.dist), list(od), flush=True)
    for pi, eps in [(1e-3, 1e-3), (1.1e-3, 1e-3), (1e-3, 1.1e-3), (5e-4, 8e-3), (0.2, 0.05), (1e-3, 1e-2)]:
        g = ctx.lynch_objective(pi, eps)
        r = O.compound_likelihood(c, pi, eps)
        print(f"  obj({pi},{eps}) gpu {g!r} oracle {r!r} rel {abs(g - r) / abs(r) if r else 0:.3e}", flush=True)
    ctx.close()
    code, hom, het, e = G.run_method(c, "likelihood_ratio", estimate_prior=True)
    rc, rcode, rhom, rhet, re_, u = O.call_method(c, "likelihood_ratio", estimate_prior=True)
    print("  est gpu", e.heterozygosity, e.error_rate, e.iterations, "oracle", re_.heterozygosity, re_.error_rate,
          re_.iterations, flush=True)
