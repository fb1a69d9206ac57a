import os, sys, json
sys.path.insert(0, ".")
import torch
import sid_amd
n = 50_000_000
dev = torch.device("cuda", 0)
counts = torch.empty((n, 4), dtype=torch.int16, device=dev)
code = torch.empty(n, dtype=torch.uint8, device=dev)
hom = torch.empty(n, dtype=torch.float64, device=dev)
het = torch.empty(n, dtype=torch.float64, device=dev)
st = torch.cuda.current_stream(dev)
ctxs = {}
for tail in ("0", "1"):
    os.environ["SID_TABLE_TAIL"] = tail
    ctxs[tail] = sid_amd.Context(0)
ctxs["0"].synth_counts(2, 30.0, 0, n, counts.data_ptr(), st.cuda_stream)
torch.cuda.synchronize()
res = {k: [] for k in ctxs}
sig = {}
for r in range(7):
    for k, c in ctxs.items():
        c.call_local(counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        if r == 0:
            sig[k] = (int(code.sum().item()), float(hom.sum().item()), float(het.sum().item()))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(10):
            c.call_local(counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st.cuda_stream)
        e.record(st)
        torch.cuda.synchronize()
        res[k].append(s.elapsed_time(e) / 10)
    # split
for k, c in ctxs.items():
    c.timing_enable(True)
    for _ in range(10):
        c.call_local(counts.data_ptr(), n, code.data_ptr(), hom.data_ptr(), het.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    c.timing_enable(False)
    print(json.dumps({"tail": k, "median_ms": sorted(res[k])[3], "min_ms": min(res[k]), "split": c.timing_read(), "sig": sig[k]}))
assert sig["0"] == sig["1"]
