"""Parity at the configs' full sizes (BASELINE.json configs[1] and [2]):
every one of the 50M sites of C2 (seed 2, -m local) and of C3 (seed 3,
-R -m likelihood_ratio) through the C ABI on the GPU against the oracle.

C3's Nelder-Mead objective sums over the whole 50M-site histogram (about 12k
unique profiles), so the trajectory -- pi-hat, eps-hat and the iteration
count, bit for bit -- is only checked for real at this size.  The -m local
oracle is per site (call.cpp:213-289 restated), so it runs on 16 shards in
parallel threads (ctypes releases the GIL); the Lynch oracle is global and
runs as one call."""
import concurrent.futures as cf

import numpy as np
import pytest

from helpers import assert_parity

pytestmark = pytest.mark.gpu

N = 50_000_000


def device_counts(sid, gpu, seed, n):
    import torch
    ctx = sid.Context(0)
    counts, code, hom, het = gpu.device_buffers(n)
    st = gpu.stream_handle(0)
    ctx.synth_counts(seed, 30.0, 0, n, counts.data_ptr(), st)
    torch.cuda.synchronize()
    return ctx, counts, code, hom, het, st


def test_c2_full_size_local(sid, gpu, oracle):
    import torch
    ctx, counts, code, hom, het, st = device_counts(sid, gpu, 2, N)
    ctx.call_local(counts.data_ptr(), N, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st)
    torch.cuda.synchronize()
    h = counts.cpu().numpy().view(np.uint16)
    # the device generator is the host generator (spot check at both ends)
    for lo in (0, N - 1000):
        assert np.array_equal(h[lo:lo + 1000], sid.synth_counts_host(2, 1000, 30.0, first=lo))
    P = 16
    cuts = [N * k // P for k in range(P + 1)]
    with cf.ThreadPoolExecutor(P) as ex:
        parts = list(ex.map(lambda k: oracle.call_local(h[cuts[k]:cuts[k + 1]]), range(P)))
    rcode = np.concatenate([p[0] for p in parts])
    rhom = np.concatenate([p[1] for p in parts])
    rhet = np.concatenate([p[2] for p in parts])
    assert_parity(code.cpu().numpy(), hom.cpu().numpy(), het.cpu().numpy(), rcode, rhom, rhet,
                  what="C2 50M sites")
    assert 45_000 < int((rcode >= 0x80).sum()) < 55_000   # ~1e-3 het sites


def test_c3_full_size_likelihood_ratio(sid, gpu, oracle):
    import torch
    _, counts, code, hom, het, st = device_counts(sid, gpu, 3, N)
    ctx = sid.Context(0, method="likelihood_ratio", estimate_prior=True)
    ctx.profile_reset(st)
    ctx.profile_accumulate(counts.data_ptr(), N, st)
    est = ctx.lynch_prepare(False)
    ctx.lookup_sites(counts.data_ptr(), N, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st)
    torch.cuda.synchronize()
    h = counts.cpu().numpy().view(np.uint16)
    rc, rcode, rhom, rhet, rest, u = oracle.call_method(h, "likelihood_ratio", estimate_prior=True)
    assert rc == 0
    assert est.n_unique == u > 10_000
    assert (est.heterozygosity, est.error_rate, est.iterations) == \
        (rest.heterozygosity, rest.error_rate, rest.iterations)
    assert_parity(code.cpu().numpy(), hom.cpu().numpy(), het.cpu().numpy(), rcode, rhom, rhet,
                  what="C3 50M sites")
