#!/usr/bin/env python3
"""bench.py — genome sites/s of sid's pileup -> CSV path on MI355X.

Headline (BASELINE.json metric, configs[1] = "C2"): 50,000,000 synthetic 30x
diploid sites per GPU, `-m local`.  A step is one whole sid run over the rank's
pileup text, already resident in HBM when the timed region starts:

    line index -> parse (counts) -> per-site call -> CSV records formatted

i.e. readFile + callSiteMLError + the output loop (call.cpp:11-20, :213-289,
sid.cpp:102-105) through the streaming engine (include/sid.h sid_engine_*,
device-text source, 128 MiB chunks); the CSV records are left in HBM.  The
PCIe-inclusive rate (text in host memory -> CSV copied back to host memory) is
reported beside it as `e2e`, and the CLI (build/sid, file -> /dev/null) as
`e2e.cli`; they are never `value`.

Configs (--config):
  C2  -m local, seed 2, 50M sites per GPU (weak scaling)           [default]
  C3  -R -m likelihood_ratio, seed 3, 50M sites per GPU (weak): ingest builds
      the profile histogram; N>1 all-gathers it over RCCL (device tensors,
      backend "nccl"), rank 0 runs the one Nelder-Mead estimate and broadcasts
      (pi, eps) over RCCL; then every rank formats its records
  C4  -m local, seed 4, 3G sites in total = 24 chromosomes x 125M (strong
      scaling: rank r takes sites [r*3G/N, (r+1)*3G/N)); the text is generated
      on the device chunk by chunk inside the step (never stored: 244 GB)
  C5  -m local, seed 5, 200x, 500M sites in total (strong), generated as C4

Multi-GPU: one rank per GPU (torchrun).  -m local has no data-path exchange;
the Lynch path exchanges only the O(U) profile histogram.  Ranks beyond the
visible GPUs are refused unless --allow-shared-gpu (a rehearsal: n_gpus then
counts distinct devices and "oversubscribed" is set).

The JSON line also carries
  roofline      the dominant kernel stage of the step (device time from HIP
                events on the engine's compute stream over the timed region),
                its algorithmic bytes per launch / average launch duration vs
                8 TB/s, and the PMC-measured HBM bytes per launch
                (profiles/pmc_<stage>_r02.json) when present
  stages_ms     device time per stage per step
  kernel_local  sid_call_local alone over resident counts (25 B/site)
  e2e           host-memory text -> CSV in host memory (PCIe both ways),
                engine clock; and the CLI on a 50M-site file
  cpu_baseline  the oracle CLI (the reference's path restated in C) on the
                same 50M-site text, 16 line-aligned shard processes, plus a
                1-core figure on a 4M-site sample (rank 0, N=1 only)
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
LOCAL_BYTES_PER_SITE = 25    # sid_call_local: 8 B counts in, 1 B code + 2 x 8 B confs out

CONFIGS = {
    "C2": dict(method="local", R=False, seed=2, depth=30.0, per_gpu=50_000_000, total=None, spc=0,
               resident=True, desc="-m local, 50M-site 30x synthetic pileup per GPU"),
    "C3": dict(method="likelihood_ratio", R=True, seed=3, depth=30.0, per_gpu=50_000_000, total=None, spc=0,
               resident=True, desc="-R -m likelihood_ratio, 50M-site 30x synthetic pileup per GPU"),
    "C4": dict(method="local", R=False, seed=4, depth=30.0, per_gpu=None, total=3_000_000_000, spc=125_000_000,
               resident=False, desc="-m local, 3G-site whole-genome 30x pileup (24 x 125M), site-range shards"),
    "C5": dict(method="local", R=False, seed=5, depth=200.0, per_gpu=None, total=500_000_000, spc=125_000_000,
               resident=False, desc="-m local, 500M-site 200x pileup, site-range shards"),
}


def parse_args():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default=None, choices=sorted(CONFIGS))
    p.add_argument("--method", default=None, choices=["local", "likelihood_ratio"],
                   help="alias: local = C2, likelihood_ratio = C3")
    p.add_argument("--sites", type=int, default=None, help="override: sites per GPU (C2/C3) or in total (C4/C5)")
    p.add_argument("--chunk-mib", type=int, default=0, help="engine chunk size (0 = 128 MiB)")
    p.add_argument("--lanes", type=int, default=1,
                   help="engine pipelines per GPU (concurrent streams; their kernels overlap, so the per-stage "
                        "event times of the roofline are only clean at 1)")
    p.add_argument("--no-extras", action="store_true", help="skip kernel_local, e2e and cpu_baseline")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--allow-shared-gpu", action="store_true",
                   help="rehearsal: more ranks than GPUs share them round-robin")
    p.add_argument("--backend", default=None, help="torch.distributed backend (default nccl = RCCL)")
    p.add_argument("--resident", action="store_true",
                   help="C4/C5: generate the rank's shard into HBM before the timed region (when it fits) "
                        "instead of on the device inside the step")
    a = p.parse_args()
    if a.config is None:
        a.config = "C3" if a.method == "likelihood_ratio" else "C2"
    return a


def stage_bytes(stage, text_per_site, csv_per_site):
    """Algorithmic HBM bytes per site of each engine stage."""
    return {
        "index": text_per_site + text_per_site / 8,    # text read once, line-start masks written
        # text read; line-start masks (1/8 of the text) and offsets read back;
        # counts (8) and the formatter's header pair (16) written
        "parse": text_per_site + text_per_site / 8 + 8 + 8 + 16,
        "call": LOCAL_BYTES_PER_SITE,                  # counts in, code + confs out
        "hist": 8,                                     # counts read
        # one-pass formatter: code + confs and the header pair read (the line
        # offset only for chrom names over 8 bytes), the records written
        "fmt_write": 17 + 16 + csv_per_site,
    }[stage]


def main():
    a = parse_args()
    cfg = dict(CONFIGS[a.config])
    gen_resident = a.resident and not cfg["resident"]   # C4/C5 shard text generated into HBM up front

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    import torch  # plumbing: device memory, events, process group
    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise SystemExit("bench.py: no HIP device visible")
    if local_rank >= ndev and not a.allow_shared_gpu:
        raise SystemExit(f"bench.py: rank {rank} (local {local_rank}) has no GPU of its own ({ndev} visible); "
                         "pass --allow-shared-gpu for a rehearsal")
    gpu = local_rank % ndev
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    n_gpus, oversub = 1, False
    if world > 1:
        import torch.distributed as dist
        backend = a.backend or "nccl"
        dist.init_process_group(backend, rank=rank, world_size=world, device_id=dev if backend == "nccl" else None)
        ids = [None] * world
        dist.all_gather_object(ids, (socket.gethostname(), gpu))
        n_gpus = len(set(ids))
        oversub = n_gpus < world
    import sid_amd

    # ---------------------------------------------------------------- input --
    if cfg["resident"]:
        n = a.sites or cfg["per_gpu"]
        first = rank * n
        total = n * world
    else:
        total = a.sites or cfg["total"]
        first, hi = total * rank // world, total * (rank + 1) // world
        n = hi - first
    text = None
    if gen_resident:
        text, ln = generate_resident(torch, sid_amd, dev, gpu, cfg, first, n)
        if not a.chunk_mib:   # 2 GiB chunks' record bounds and hold arena overran the HBM the text leaves (C4, 1 GPU)
            a.chunk_mib = 1024
        cfg["resident"] = True
        cfg["desc"] += "; the shard's text generated into HBM before the timed region"
    elif cfg["resident"]:
        ctx = sid_amd.Context(gpu)
        cap = int(n * (24 + 2.9 * cfg["depth"])) + (64 << 20)
        text = torch.empty(cap + 512, dtype=torch.uint8, device=dev)
        ln = ctx.synth_text_device(cfg["seed"], cfg["depth"], first, n, text.data_ptr(), cap,
                                   sites_per_chrom=cfg["spc"])
        text[ln:ln + 512].zero_()
        torch.cuda.synchronize(dev)
        ctx.close()
    lynch = cfg["method"] != "local" or cfg["R"]
    # one pipeline per GPU: with 2 GiB chunks a second one measured no gain
    # for -m local (5.50-5.54 vs 5.51-5.59 ms/step) and a loss for the Lynch
    # paths (per-chunk histogram syncs, the lanes' table merge: C3 6.95 ->
    # 8.51 ms), whose multi-rank exchange also reads one context
    lanes = 1 if lynch else max(1, a.lanes)
    eng = sid_amd.Engine(method=cfg["method"], estimate_prior=cfg["R"], devices=1, first_device=gpu,
                         chunk_bytes=a.chunk_mib << 20, device_sink=1, lanes=lanes)
    if cfg["resident"]:
        eng.source_device_text(text.data_ptr(), ln, keep=text)
    else:
        eng.source_synth(cfg["seed"], n, cfg["depth"], first=first, sites_per_chrom=cfg["spc"], on_device=True)
    est_box = {}

    def step():
        st = eng.ingest()
        if lynch and dist is not None:
            exchange_histogram(torch, dist, eng, dev, rank)
        if lynch and dist is not None and world > 1:
            est = broadcast_estimate(torch, dist, eng, dev, rank)
        else:
            est = eng.estimate()
        _, st2 = eng.emit()
        est_box["est"] = est
        return st, st2

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    eng.profile(True)   # HIP event pairs around every stage on the compute stream
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st, st2 = step()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    prof = eng.profile_read()
    eng.profile(False)
    sites_rank = st.sites
    stages = {k[:-3]: v / a.steps for k, v in prof.items() if k.endswith("_ms") and k != "fmt_len_ms"}
    if dist:
        vec = torch.tensor([elapsed] + [stages[k] for k in sorted(stages)], dtype=torch.float64, device=dev)
        dist.all_reduce(vec, op=dist.ReduceOp.MAX)
        elapsed = float(vec[0])
        stages = {k: float(v) for k, v in zip(sorted(stages), vec[1:].tolist())}
        tot = torch.tensor([float(sites_rank)], dtype=torch.float64, device=dev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        sites_all = int(tot.item())
    else:
        sites_all = sites_rank

    if rank == 0:
        text_bytes = st.bytes_in if cfg["resident"] else None
        tps = (text_bytes / sites_rank) if text_bytes else (24 + 2.7 * cfg["depth"])
        cps = st2.bytes_out / sites_rank if sites_rank else 0.0
        dom = max(stages, key=lambda k: stages[k])
        bps = stage_bytes(dom, tps, cps)
        per_launch_sites = sites_rank / max(1, prof["chunks"] / a.steps)
        launch_ms = stages[dom] / max(1, prof["chunks"] / a.steps)
        achieved = bps * per_launch_sites / (launch_ms * 1e-3) / 1e9
        traffic = pmc_traffic(dom, per_launch_sites)
        step_bytes = (text_bytes or 0) + st2.bytes_out
        out = {
            "metric": "genome sites/sec (whole node) on 30x synthetic pileup; 1/2/4/8 GPU scaling",
            "value": sites_all * a.steps / elapsed,
            "unit": "sites/s",
            "n_gpus": n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if cfg["total"] else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (counter-based pileup generator, BASELINE.md): pileup text "
                     + ("resident in HBM before the timed region" + (" (the rank's shard of the fixed total, "
                                                                      "generated in 50M-site pieces)"
                                                                      if gen_resident else "")
                        if cfg["resident"] else
                        "generated on the device chunk by chunk inside the step (never stored)")
                     + "; CSV records formatted into HBM"),
            "config": {"workload": f"{a.config}: {cfg['desc']}", "method": cfg["method"],
                       "estimate_prior": cfg["R"], "seed": cfg["seed"], "depth": cfg["depth"],
                       "sites_per_gpu": n, "sites_total": sites_all,
                       "sites_per_chrom": cfg["spc"] or None, "chunks_per_step_rank0": prof["chunks"] / a.steps,
                       "text_bytes_rank0": text_bytes, "csv_bytes_rank0": st2.bytes_out,
                       "parallelism": f"site-range shards x{world}" + (" + RCCL histogram all-gather"
                                                                       if lynch and world > 1 else ""),
                       "ranks": world, "oversubscribed": oversub, "engine_lanes_per_gpu": lanes},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": f"engine stage '{dom}'", "stage_kernels": STAGE_KERNELS[dom],
                         "launch_ms": launch_ms, "sites_per_launch": per_launch_sites,
                         "bytes_per_site": bps, "valu": valu_issue(dom, per_launch_sites, launch_ms)},
            "stages_ms": stages,
            "path": {"bytes_per_site": tps + cps, "text_per_site": tps, "csv_per_site": cps,
                     "GBps": step_bytes / (elapsed / a.steps) / 1e9 if text_bytes else None,
                     "note": "text in + CSV out per step (the path's minimum HBM traffic) / ms_per_step"},
        }
        if lynch:
            e = est_box["est"]
            out["estimate"] = {"pi": e.heterozygosity, "eps": e.error_rate, "iterations": e.iterations,
                               "n_unique": e.n_unique}
        if world == 1 and cfg["resident"] and not gen_resident and not a.no_extras:
            out["kernel_local"] = bench_kernel_local(torch, dev, cfg, n)
            out["e2e"] = bench_e2e(torch, sid_amd, cfg, text, ln, n, a)
            if not a.no_cpu:
                out["cpu_baseline"] = bench_cpu(cfg, text, ln, n)
        print(json.dumps(out), flush=True)
    eng.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


STAGE_KERNELS = {
    "index": ["sid_index_count_kernel", "sid_scan_*"],
    "parse": ["sid_index_emit_kernel", "sid_parse_kernel", "sid_parse_serial_kernel"],
    "call": ["sid_local_table_p2", "sid_local_fixup"],
    "hist": ["sid_hist_dense_kernel", "sid_hist_reduce_kernel"],
    "fmt_write": ["sid_fmt_fused_kernel"],
}


VALU_ISSUE_PER_S = 256 * 4 / 2 * 2.4e9   # wave64 VALU instructions/s: 1024 SIMDs, one per 2 cycles, 2.4 GHz


def valu_issue(stage, sites, launch_ms):
    """The stage's VALU work against the chip's VALU issue rate: SQ_INSTS_VALU
    per site of its kernels (profiles/pmc_c2_r02_summary.json, the committed
    PMC pass of tools/gpu_pmc_c2.sh) x the sites of a launch, at one wave64
    instruction per SIMD per 2 cycles (MI355X_MICROARCH.md); None when absent."""
    try:
        pm = json.load(open(os.path.join(ROOT, "profiles", "pmc_c2_r02_summary.json")))
        sites_pmc = json.load(open(os.path.join(ROOT, "profiles", f"pmc_{stage}_r02.json")))["sites_per_launch"]
    except Exception:
        return None
    insts = 0.0
    for k in STAGE_KERNELS[stage]:
        for name, r in pm.items():
            if name.startswith(k.rstrip("*")) and "SQ_INSTS_VALU" in r:
                insts += r["SQ_INSTS_VALU"] / sites_pmc
    if not insts:
        return None
    per_launch = insts * sites
    issue_ms = per_launch / VALU_ISSUE_PER_S * 1e3
    return {"insts_per_launch": per_launch, "issue_bound_ms": issue_ms, "frac": issue_ms / launch_ms,
            "note": "VALU instructions of the stage's kernels (PMC) at the chip's issue rate vs the measured launch"}


def pmc_traffic(stage, sites):
    """HBM bytes per launch of the stage from the committed PMC summary
    (tools/pmc_traffic.py over separate FETCH_SIZE / WRITE_SIZE passes), scaled
    to this launch's sites; None when absent."""
    p = os.path.join(ROOT, "profiles", f"pmc_{stage}_r02.json")
    try:
        pm = json.load(open(p))
        return pm["hbm_bytes_per_site"] * sites
    except Exception:
        return None


def generate_resident(torch, sid_amd, dev, gpu, cfg, first, n):
    """The rank's shard of C4/C5 as text in HBM: one buffer sized to the
    text (the rest, at least a 24 GiB reserve, stays free for the engine's
    chunk workspace, pooled record buffers and hold arena), filled by the device generator in 50M-site pieces
    laid end to end (every line stands alone, so the pieces concatenate to the
    shard's text); refuses a shard that does not fit."""
    free, _ = torch.cuda.mem_get_info(dev)
    reserve = 24 << 30
    cap = free - reserve
    need = int(n * (2.72 * cfg["depth"] + 2))   # ~81 B/site at 30x, ~564 at 200x (measured)
    if cap < need:
        raise SystemExit(f"bench.py --resident: the shard's ~{need / 1e9:.0f} GB of text does not fit "
                         f"({free / 1e9:.0f} GB free, {reserve >> 30} GiB kept for the engine)")
    cap = min(cap, int(need * 1.03) + (1 << 30))   # the rest stays free for the engine
    text = torch.empty(cap, dtype=torch.uint8, device=dev)
    ctx = sid_amd.Context(gpu)
    ln, piece = 0, 50_000_000
    for lo in range(0, n, piece):
        m = min(piece, n - lo)
        ln += ctx.synth_text_device(cfg["seed"], cfg["depth"], first + lo, m, text.data_ptr() + ln,
                                    cap - 512 - ln, sites_per_chrom=cfg["spc"])
    text[ln:ln + 512].zero_()
    torch.cuda.synchronize(dev)
    ctx.close()
    return text, ln


def exchange_histogram(torch, dist, eng, dev, rank):
    """The one exchange of the Lynch path: every rank's unique-profile table
    (O(U) x 16 B) all-gathered as device tensors over RCCL, merged, loaded."""
    from sid_amd import dist as sdist
    ctx = sid_amd_ctx(eng)
    keys, cnts = ctx.profile_table()
    keys, cnts = sdist.allgather_profile_table(keys, cnts, device=dev)
    ctx.profile_load(keys, cnts)


def broadcast_estimate(torch, dist, eng, dev, rank):
    """Rank 0 runs the one Nelder-Mead estimate on the merged table; (pi, eps)
    go to the other ranks over RCCL, which classify with them."""
    import sid_amd
    if rank == 0:
        est = eng.estimate()
        vec = torch.tensor([est.heterozygosity, est.error_rate, float(est.iterations)], dtype=torch.float64,
                           device=dev)
    else:
        vec = torch.zeros(3, dtype=torch.float64, device=dev)
    dist.broadcast(vec, 0)
    if rank != 0:
        g = sid_amd.Estimate()
        g.heterozygosity, g.error_rate, g.iterations = float(vec[0]), float(vec[1]), int(vec[2])
        est = eng.estimate(given=g)
    return est


def sid_amd_ctx(eng):
    import sid_amd
    return sid_amd.Context.wrap(eng.context(0))


def bench_kernel_local(torch, dev, cfg, n):
    """sid_call_local alone over the counts of the same sites resident in HBM
    (the per-site arithmetic kernel: 25 B/site), HIP events on its stream."""
    import sid_amd
    ctx = sid_amd.Context(dev.index)
    st = torch.cuda.current_stream(dev)
    counts = torch.empty((n, 4), dtype=torch.int16, device=dev)
    code = torch.empty(n, dtype=torch.uint8, device=dev)
    hom = torch.empty(n, dtype=torch.float64, device=dev)
    het = torch.empty(n, dtype=torch.float64, device=dev)
    ctx.synth_counts(cfg["seed"], cfg["depth"], 0, n, counts.data_ptr(), st.cuda_stream)
    args = (counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st.cuda_stream)
    for _ in range(3):
        ctx.call_local(*args)
    torch.cuda.synchronize(dev)
    K = 20
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for s, e in ev:
        s.record(st)
        ctx.call_local(*args)
        e.record(st)
    torch.cuda.synchronize(dev)
    ms = sum(s.elapsed_time(e) for s, e in ev) / K
    ctx.timing_enable(True)
    for _ in range(10):
        ctx.call_local(*args)
    torch.cuda.synchronize(dev)
    ctx.timing_enable(False)
    _, main_ms, fix_ms = ctx.timing_read()
    ctx.close()
    gbs = LOCAL_BYTES_PER_SITE * n / (ms * 1e-3) / 1e9
    pm = None
    try:
        pm = json.load(open(os.path.join(ROOT, "profiles", "pmc_local_r01.json"))).get("hbm_bytes_per_launch")
    except Exception:
        pass
    return {"sites_per_s": n / (ms * 1e-3), "ms": ms, "GBps": gbs, "frac": gbs / HBM_PEAK_GBS,
            "split_ms": {"sid_local_table_p2": main_ms, "sid_local_fixup": fix_ms}, "bytes_per_site": 25,
            "traffic": pm, "note": "counts resident in HBM -> code + confs (the round-1 headline kernel)"}


def bench_e2e(torch, sid_amd, cfg, text, ln, n, a):
    """PCIe-inclusive: (1) the engine over the text in pinned host memory, CSV
    copied back into pinned host memory (engine clock); (2) the CLI on the same
    text as a file in the page cache, CSV to /dev/null (wall clock and the
    CLI's own clock)."""
    res = {"sites": n, "text_bytes": ln}
    host = text[:ln].cpu().pin_memory()
    eng = sid_amd.Engine(method=cfg["method"], estimate_prior=cfg["R"], device_sink=2,
                         chunk_bytes=a.chunk_mib << 20)
    eng.source_host_ptr(host.data_ptr(), ln, keep=host)
    runs = []
    for r in range(3):
        t0 = time.perf_counter()
        st = eng.ingest()
        eng.estimate()
        _, st2 = eng.emit()
        runs.append(time.perf_counter() - t0)
    eng.close()
    dt = min(runs[1:])
    res["host_memory"] = {"sites_per_s": n / dt, "s": dt, "runs_s": runs, "csv_bytes": st2.bytes_out,
                          "note": "pinned host text -> H2D -> index/parse/call/format -> D2H into pinned host "
                                  "memory (records dropped there), one GPU, engine clock"}
    del host
    cli = os.path.join(ROOT, "build", "sid")
    if not os.path.exists(cli):
        return res
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "c.plp")
        write_text_file(text, ln, path)
        flags = [] if cfg["method"] == "local" else (["-R"] if cfg["R"] else []) + ["-m", cfg["method"]]
        cli_runs = []
        for _ in range(3):
            with open(os.devnull, "wb") as dn:
                t0 = time.perf_counter()
                r = subprocess.run([cli, "--stats"] + flags + [path], stdout=dn, stderr=subprocess.PIPE)
                dt = time.perf_counter() - t0
            if r.returncode != 0:
                res["cli"] = {"error": r.returncode, "stderr": r.stderr.decode()[-400:]}
                return res
            try:
                stt = json.loads(r.stderr.decode().strip().splitlines()[-1])
            except Exception:
                stt = {}
            cli_runs.append((dt, stt))
        dt, stt = min(cli_runs[1:], key=lambda x: x[0])
        res["cli"] = {"wall_s": dt, "sites_per_s_wall": n / dt, "sites_per_s_cli_clock": stt.get("sites_per_s"),
                      "wall_s_runs": [x[0] for x in cli_runs], "cli_stats": stt,
                      "note": "build/sid FILE > /dev/null, one GPU: wall = process start + HIP init + mmap + "
                              "H2D + parse/call/format + D2H + write; cli_clock = input mapping to last write"}
    return res


def write_text_file(text, ln, path):
    """The resident text, copied back in 256 MiB pieces, as a file."""
    step = 256 << 20
    with open(path, "wb") as f:
        for lo in range(0, ln, step):
            f.write(text[lo:min(ln, lo + step)].cpu().numpy().tobytes())
    with open(path, "rb") as f:   # into the page cache
        while f.read(1 << 26):
            pass


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def bench_cpu(cfg, text, ln, n):
    """The oracle CLI (reference sid.cpp/call.cpp/lynch/stats restated in C,
    single-threaded) on the same text: 16 line-aligned shard processes over
    all n sites (-m local: sites are independent; the GPU box's CPU share is
    16 cores), and one process on the first 4M sites."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    if not os.path.exists(oracle.CLI):
        oracle.build()
    flags = [] if cfg["method"] == "local" else (["-R"] if cfg["R"] else []) + ["-m", cfg["method"]]
    P = 16
    host = text[:ln].cpu().numpy()
    with tempfile.TemporaryDirectory() as td:
        cuts = [0]
        for k in range(1, P):
            c = ln * k // P
            nl = host[c:c + (1 << 20)].tobytes().find(b"\n")
            cuts.append(c + nl + 1)
        cuts.append(ln)
        paths = []
        for k in range(P):
            pth = os.path.join(td, f"s{k}.plp")
            with open(pth, "wb") as f:
                f.write(host[cuts[k]:cuts[k + 1]].tobytes())
            paths.append(pth)
        res = {"unit": "sites/s", "kind": "port", "cpu_model": cpu_model()}
        if cfg["method"] == "local":
            with open(os.devnull, "wb") as dn:
                t0 = time.perf_counter()
                procs = [subprocess.Popen([oracle.CLI] + flags + [p], stdout=dn, stderr=subprocess.DEVNULL)
                         for p in paths]
                rcs = [p.wait() for p in procs]
                dt = time.perf_counter() - t0
            res.update({"value": n / dt if not any(rcs) else None, "cores": P, "seconds": dt,
                        "sample": f"the same {n:,}-site {cfg['desc']} text ({ln / 1e9:.2f} GB), {P} line-aligned "
                                  f"shards, one oracle/_build/sid_oracle process each, CSV to /dev/null, wall"})
        # one core on the first 4M sites
        m = min(n, 4_000_000)
        cut = 0
        need = m
        while need > 0:
            nl = host[cut:cut + (64 << 20)].tobytes().count(b"\n")
            if nl <= need:
                cut += 64 << 20
                need -= nl
            else:
                seg = host[cut:cut + (64 << 20)].tobytes()
                idx = -1
                for _ in range(need):
                    idx = seg.find(b"\n", idx + 1)
                cut += idx + 1
                need = 0
        one = os.path.join(td, "one.plp")
        with open(one, "wb") as f:
            f.write(host[:cut].tobytes())
        with open(os.devnull, "wb") as dn:
            t0 = time.perf_counter()
            r = subprocess.run([oracle.CLI] + flags + [one], stdout=dn, stderr=subprocess.DEVNULL)
            dt = time.perf_counter() - t0
        single = {"value": m / dt if r.returncode == 0 else None, "cores": 1, "seconds": dt,
                  "sample": f"the first {m:,} sites of the same text, one process"}
        if "value" not in res:
            res.update(single)
            res["sample"] = single["sample"]
        else:
            res["single_core"] = single
    return res


if __name__ == "__main__":
    main()
