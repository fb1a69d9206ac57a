#!/usr/bin/env python3
"""bench.py — genome sites/s of the sid hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): 50,000,000 synthetic 30x diploid
sites per GPU, `-m local`.  A step is one pass of the hot path
(sid_call_local: counts -> code + hom_conf + het_conf) over one batch of 50M
sites already resident in HBM.  N GPUs = N ranks (torchrun), each with its own
50M-site range of the counter-based generator (weak scaling, no data-path
collective; gloo only for the barrier and the max over ranks).

With --method likelihood_ratio (BASELINE configs[2], "C3": the reference has
no `-m lynch`; SURVEY.md §8(d) runs C3 as `-R -m likelihood_ratio`), a step is
the whole Lynch path over the resident 50M sites: profile histogram (device
hash), [N>1: one all-gather of the histograms], Nelder-Mead on the GPU
objective, classification + Benjamini-Hochberg, and the per-site lookup.
`--method bayes` runs the same with the posterior classification.

Prints ONE JSON line on rank 0 (contract in the task statement), including
  roofline      25 algorithmic bytes/site (8 B counts in, 1 B code + 2 x 8 B
                confs out) / average kernel duration from HIP events on the
                launch stream, against 8 TB/s HBM3E;
  cpu_baseline  the oracle's end-to-end CLI (reference sid.cpp/call.cpp
                restated in C, single thread, text -> CSV) on a bounded sample
                of the same workload, rank 0 at N=1 only;
  e2e           the product CLI (build/sid) on the same sample file, text
                in -> CSV out, device text path and --host-parse (wall clock
                of the whole process and the CLI's own clock), informational;
  pipeline      SURVEY.md §8(d) throughput 2: counts in pinned host memory ->
                H2D -> sid_call_local -> D2H of code + confs, in chunks over
                three streams (PCIe-bound, 25 B/site cross the link),
                informational.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BYTES_PER_SITE = 25          # 8 in + 17 out
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--sites", type=int, default=50_000_000, help="sites per GPU")
    p.add_argument("--depth", type=float, default=30.0)
    p.add_argument("--seed", type=int, default=None, help="default: 2 (C2) / 3 (C3)")
    p.add_argument("--cpu-sample", type=int, default=16_000_000,
                   help="sites in the CPU-baseline / e2e sample (0 = skip); ~10 s of oracle CPU time at C2")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--method", default="local", choices=["local", "likelihood_ratio", "bayes"],
                   help="local = C2 (default); likelihood_ratio = C3 (with -R, as SURVEY.md §8(d)); bayes")
    p.add_argument("--no-R", action="store_true", help="C3 without -R (estimate_prior off)")
    p.add_argument("--direct", action="store_true",
                   help="A/B: bypass the class-table kernel (SID_LOCAL_DIRECT=1)")
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_local_r01.json"),
                   help="per-launch HBM traffic from a rocprofv3 --pmc pass (tools/pmc_traffic.py)")
    return p.parse_args()


def main():
    a = parse_args()
    if a.seed is None:
        a.seed = 2 if a.method == "local" else 3
    if a.direct:
        os.environ["SID_LOCAL_DIRECT"] = "1"
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    import torch  # plumbing: device memory, streams, events, process group
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import sid_amd
    # one rank per GPU; more ranks than GPUs share them round-robin (a
    # rehearsal of the N>1 path on a smaller box)
    gpu = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    n = a.sites
    ctx = sid_amd.Context(gpu)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    counts = torch.empty((n, 4), dtype=torch.int16, device=dev)
    code = torch.empty(n, dtype=torch.uint8, device=dev)
    hom = torch.empty(n, dtype=torch.float64, device=dev)
    het = torch.empty(n, dtype=torch.float64, device=dev)
    # inputs resident in HBM before the timed region: this rank's site range
    ctx.synth_counts(a.seed, a.depth, rank * n, n, counts.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    if a.method != "local":
        ctx.close()
        return bench_lynch(a, torch, dist, rank, world, dev, counts, code, hom, het)

    def step():
        ctx.call_local(counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), sh)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # HIP events on the launch stream bracket every step of the timed region;
    # a step is one sid_call_local = class-table kernel + fix-up kernel
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.steps)]
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    step_ms = sum(s.elapsed_time(e) for s, e in ev) / a.steps
    # split of a step into its two kernels, from libsid's own events in a
    # separate untimed pass (events between the kernels would perturb the
    # timed region)
    ctx.timing_enable(True)
    for _ in range(min(a.steps, 10)):
        step()
    torch.cuda.synchronize(dev)
    ctx.timing_enable(False)
    ncalls, main_ms, fixup_ms = ctx.timing_read()
    if dist:
        t = torch.tensor([elapsed, step_ms, main_ms, fixup_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, step_ms, main_ms, fixup_ms = (float(x) for x in t)

    # a cheap on-device sanity check of this rank's last step (host oracle
    # parity is covered by tests/ and smoke())
    nhet = int((code >= 0x80).sum().item())

    if rank == 0:
        value = world * n * a.steps / elapsed
        # the unit priced against the roofline is the whole sid_call_local
        # (class-table kernel + fix-up), timed over the timed region
        kern_ms = step_ms
        achieved = BYTES_PER_SITE * n / (kern_ms * 1e-3) / 1e9
        traffic = None
        if a.pmc_json and os.path.exists(a.pmc_json):
            try:
                pm = json.load(open(a.pmc_json))
                if int(pm.get("sites", -1)) == n:
                    traffic = pm.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": "genome sites/sec (whole node) on 30x synthetic pileup; 1/2/4/8 GPU scaling",
            "value": value,
            "unit": "sites/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (counter-based 30x diploid pileup generator, BASELINE.md), counts resident in HBM",
            "config": {"workload": "C2: -m local, 50M-site 30x synthetic pileup per GPU",
                       "sites_per_gpu": n, "depth": a.depth, "seed": a.seed, "method": "local",
                       "parallelism": f"site-range shards x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": ("sid_call_local = sid_local_table_p2 + sid_local_fixup" if not a.direct
                                    else "sid_local_kernel_x4"),
                         "kernel_ms": kern_ms, "bytes_per_site": BYTES_PER_SITE,
                         "split_ms": {"sid_local_table_p2": main_ms, "sid_local_fixup": fixup_ms},
                         "achieved_main_kernel": (BYTES_PER_SITE * n / (main_ms * 1e-3) / 1e9
                                                  if main_ms > 0 else None)},
            "het_sites_last_step": nhet,
            "kernel_path": "direct" if a.direct else "class-table + fix-up",
        }
        if world == 1 and not a.no_e2e:
            out["pipeline"] = bench_pipeline(a, torch, dev, counts, code, hom, het)
        if world == 1 and a.cpu_sample > 0:
            out["cpu_baseline"], e2e = cpu_and_e2e(a)
            if e2e is not None:
                out["e2e"] = e2e
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def bench_pipeline(a, torch, dev, counts, code, hom, het):
    """Pinned host counts -> H2D -> sid_call_local -> D2H (code, hom, het) for
    the whole shard, 4M-site chunks round-robin over three streams, one
    context per stream (a context's miss list is per call)."""
    import sid_amd
    n = a.sites
    chunk = 1 << 22
    nstreams = 3
    h_counts = counts.cpu().pin_memory()
    h_code = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_hom = torch.empty(n, dtype=torch.float64).pin_memory()
    h_het = torch.empty(n, dtype=torch.float64).pin_memory()
    lanes = []
    for _ in range(nstreams):
        lanes.append((torch.cuda.Stream(dev), sid_amd.Context(dev.index),
                      torch.empty((chunk, 4), dtype=torch.int16, device=dev),
                      torch.empty(chunk, dtype=torch.uint8, device=dev),
                      torch.empty(chunk, dtype=torch.float64, device=dev),
                      torch.empty(chunk, dtype=torch.float64, device=dev)))

    def run():
        for k, lo in enumerate(range(0, n, chunk)):
            s, cx, dc, dcode, dhom, dhet = lanes[k % nstreams]
            m = min(chunk, n - lo)
            with torch.cuda.stream(s):
                dc[:m].copy_(h_counts[lo:lo + m], non_blocking=True)
                cx.call_local(dc.data_ptr(), m, dcode.data_ptr(), dhom.data_ptr(), dhet.data_ptr(), s.cuda_stream)
                h_code[lo:lo + m].copy_(dcode[:m], non_blocking=True)
                h_hom[lo:lo + m].copy_(dhom[:m], non_blocking=True)
                h_het[lo:lo + m].copy_(dhet[:m], non_blocking=True)
        torch.cuda.synchronize(dev)

    run()
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        run()
        times.append(time.perf_counter() - t0)
    # the same outputs as the resident run (bit patterns, NaN-safe)
    ok = (torch.equal(h_code, code.cpu()) and torch.equal(h_hom.view(torch.int64), hom.cpu().view(torch.int64))
          and torch.equal(h_het.view(torch.int64), het.cpu().view(torch.int64)))
    for _, cx, *_ in lanes:
        cx.close()
    dt = min(times)
    return {"value": n / dt, "unit": "sites/s", "seconds": dt, "runs_s": times, "chunk_sites": chunk,
            "streams": nstreams, "pcie_GBps": 25 * n / dt / 1e9, "equals_resident_run": ok,
            "note": "pinned host counts -> H2D -> sid_call_local -> D2H of code + hom + het (25 B/site over PCIe)"}


LYNCH_HIST_BYTES = 8         # histogram pass reads the counts
LYNCH_LOOKUP_BYTES = 25      # lookup pass: 8 in + 17 out


def bench_lynch(a, torch, dist, rank, world, dev, counts, code, hom, het):
    """C3: the whole -R -m likelihood_ratio (or bayes) path per step."""
    import sid_amd
    from sid_amd import dist as sdist
    n = a.sites
    R = not a.no_R
    ctx = sid_amd.Context(dev.index, method=a.method, estimate_prior=R)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    cp = counts.data_ptr()
    ev = []

    def step(record):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if record else None
        t0 = time.perf_counter()
        if e:
            e[0].record(stream)
        ctx.profile_reset(sh)
        ctx.profile_accumulate(cp, n, sh)
        if e:
            e[1].record(stream)
        if world > 1:   # the one exchange of the Lynch path: O(U) histogram
            keys, cnts = ctx.profile_table()
            keys, cnts = sdist.allgather_profile_table(keys, cnts)
            ctx.profile_load(keys, cnts)
        t1 = time.perf_counter()
        est = ctx.lynch_prepare(False)
        t2 = time.perf_counter()
        if e:
            e[2].record(stream)
        ctx.lookup_sites(cp, n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), sh)
        if e:
            e[3].record(stream)
            ev.append((e, t1 - t0, t2 - t1))
        return est

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        est = step(True)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    hist_ms = sum(e[0].elapsed_time(e[1]) for e, _, _ in ev) / a.steps
    look_ms = sum(e[2].elapsed_time(e[3]) for e, _, _ in ev) / a.steps
    prep_ms = sum(p for _, _, p in ev) / a.steps * 1e3
    if dist:
        t = torch.tensor([elapsed, hist_ms, look_ms, prep_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, hist_ms, look_ms, prep_ms = (float(x) for x in t)
    nhet = int((code >= 0x80).sum().item())
    u = len(ctx.profile_table()[0])
    if rank == 0:
        hist_gbs = LYNCH_HIST_BYTES * n / (hist_ms * 1e-3) / 1e9
        look_gbs = LYNCH_LOOKUP_BYTES * n / (look_ms * 1e-3) / 1e9
        dom = ("sid_lookup_sites", look_gbs, look_ms) if look_ms >= hist_ms else \
              ("sid_profile_accumulate", hist_gbs, hist_ms)
        out = {
            "metric": "genome sites/sec (whole node) on 30x synthetic pileup; 1/2/4/8 GPU scaling",
            "value": world * n * a.steps / elapsed,
            "unit": "sites/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (counter-based 30x diploid pileup generator, BASELINE.md), counts resident in HBM",
            "config": {"workload": f"C3: {'-R ' if R else ''}-m {a.method}, 50M-site 30x synthetic pileup per GPU",
                       "sites_per_gpu": n, "depth": a.depth, "seed": a.seed, "method": a.method,
                       "estimate_prior": R, "parallelism": f"site-range shards x{world} + histogram all-gather"},
            "roofline": {"bound": "hbm", "achieved": dom[1], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": dom[1] / HBM_PEAK_GBS, "traffic": None, "kernel": dom[0], "kernel_ms": dom[2],
                         "kernels": {"sid_profile_accumulate": {"ms": hist_ms, "bytes_per_site": LYNCH_HIST_BYTES,
                                                                "GBps": hist_gbs},
                                     "sid_lookup_sites": {"ms": look_ms, "bytes_per_site": LYNCH_LOOKUP_BYTES,
                                                          "GBps": look_gbs}}},
            "phases_ms": {"histogram": hist_ms, "estimate_classify_host": prep_ms, "lookup": look_ms},
            "estimate": {"pi": est.heterozygosity, "eps": est.error_rate, "iterations": est.iterations,
                         "evaluations": est.evaluations, "unique_profiles": u},
            "het_sites_last_step": nhet,
        }
        if world == 1 and not a.no_e2e:
            out["pipeline"] = bench_pipeline(a, torch, dev, counts, code, hom, het)
        if world == 1 and a.cpu_sample > 0:
            out["cpu_baseline"], e2e = cpu_and_e2e(a)
            if e2e is not None:
                out["e2e"] = e2e
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def method_flags(a):
    if a.method == "local":
        return []
    return (["-R"] if not a.no_R else []) + ["-m", a.method]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_sharded(a, td, cli):
    """the CPU path with one process per core on line-aligned
    shards of the same sample (valid for -m local: sites are independent),
    P = min(16, cpu_count) -- the GPU box's CPU share is 16 cores."""
    import sid_amd
    P = max(1, min(16, os.cpu_count() or 1))
    m = a.cpu_sample
    paths = []
    for k in range(P):
        lo, hi = m * k // P, m * (k + 1) // P
        pth = os.path.join(td, f"shard{k}.plp")
        with open(pth, "wb") as f:
            f.write(sid_amd.synth_text(a.seed, hi - lo, a.depth, first=lo))
        with open(pth, "rb") as f:
            while f.read(1 << 26):
                pass
        paths.append(pth)
    with open(os.devnull, "wb") as dn:
        t0 = time.perf_counter()
        procs = [subprocess.Popen([cli] + method_flags(a) + [pth], stdout=dn, stderr=subprocess.DEVNULL)
                 for pth in paths]
        rcs = [pr.wait() for pr in procs]
        dt = time.perf_counter() - t0
    for pth in paths:
        os.unlink(pth)
    return {"value": m / dt if not any(rcs) else None, "unit": "sites/s", "cores": P, "seconds": dt,
            "note": f"{P} oracle processes on line-aligned shards of the same {m:,}-site sample, wall clock"}


def cpu_and_e2e(a):
    """Oracle CLI (reference path restated, 1 thread) and the product CLI on the
    same bounded sample text of the workload (file in page cache, CSV to
    /dev/null).  The product runs twice: the device text path (text to HBM,
    parsed and formatted on the GPU) and --host-parse."""
    import sid_amd
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    m = a.cpu_sample
    base = None
    e2e = None
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "sample.plp")
        with open(path, "wb") as f:
            step = 2_000_000
            for lo in range(0, m, step):
                f.write(sid_amd.synth_text(a.seed, min(step, m - lo), a.depth, first=lo))
        size = os.path.getsize(path)
        if not os.path.exists(oracle.CLI):
            oracle.build()
        with open(path, "rb") as f:   # page cache
            while f.read(1 << 26):
                pass
        t0 = time.perf_counter()
        with open(os.devnull, "wb") as dn:
            r = subprocess.run([oracle.CLI] + method_flags(a) + [path], stdout=dn, stderr=subprocess.PIPE)
        dt = time.perf_counter() - t0
        base = {"value": m / dt if r.returncode == 0 else None, "unit": "sites/s", "cores": 1,
                "kind": "port",
                "sample": f"{m:,} sites of the {'C2' if a.method == 'local' else 'C3'} generator "
                          f"{' '.join(method_flags(a))} (seed {a.seed}, {a.depth:g}x, {size / 1e9:.2f} GB text), "
                          f"pileup text -> CSV to /dev/null, oracle/_build/sid_oracle "
                          f"(call.cpp/lynch.hpp/stats.cpp restated, single thread), {dt:.2f} s",
                "cpu_model": cpu_model()}
        if a.method == "local" and r.returncode == 0:
            base["sharded"] = cpu_sharded(a, td, oracle.CLI)
        if not a.no_e2e and os.path.exists(sid_amd.CLI_PATH):
            e2e = {"unit": "sites/s", "sites": m, "text_bytes": size,
                   "note": "build/sid on the sample file: wall clock of the whole process (start, HIP init, "
                           "mmap, text -> HBM over PCIe, parse, call, CSV formatting, D2H, write to /dev/null); "
                           "in_process = the CLI's own clock from input mapping to the last byte written"}
            for tag, extra in (("device_text_path", []), ("host_parse", ["--host-parse"])):
                runs = []
                for _ in range(2):   # the first run of a fresh process on the box also loads code objects
                    with open(os.devnull, "wb") as dn:
                        t0 = time.perf_counter()
                        r = subprocess.run([sid_amd.CLI_PATH, "--stats"] + extra + method_flags(a) + [path],
                                           stdout=dn, stderr=subprocess.PIPE)
                        dt = time.perf_counter() - t0
                    if r.returncode != 0:
                        runs = None
                        e2e[tag] = {"error": r.returncode}
                        break
                    try:
                        st = json.loads(r.stderr.decode().strip().splitlines()[-1])
                    except Exception:
                        st = {}
                    runs.append((dt, st))
                if not runs:
                    continue
                dt, st = min(runs, key=lambda x: x[0])
                e2e[tag] = {"wall_s": dt, "value_wall": m / dt, "value_in_process": st.get("sites_per_s"),
                            "wall_s_runs": [x[0] for x in runs], "cli_stats": st}
    return base, e2e


if __name__ == "__main__":
    main()
