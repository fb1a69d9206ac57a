# Context creation time (class tables built per context) -- measurement only
import time, sys
sys.path.insert(0, ".")
import sid_amd, torch
torch.cuda.init()
c = sid_amd.Context(0); torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    c = sid_amd.Context(0)
torch.cuda.synchronize()
print("context create ms", (time.perf_counter() - t) / 20 * 1e3)
