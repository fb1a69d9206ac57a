"""The CLI (build/sid FILE > /dev/null) on the 50M-site C2 text under copy
engine settings and CLI options: wall and the CLI's own clock per run."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from sid_amd import gpu as G  # noqa: E402
import bench  # noqa: E402

text, ln = G.synth_text_hbm(2, 30.0, 0, 50_000_000, device=0)
path = "/tmp/c2.plp"
bench.write_text_file(text, ln, path)
del text
torch.cuda.empty_cache()
cli = os.path.join(ROOT, "build", "sid")
variants = [("sdma1", {"HSA_ENABLE_SDMA": "1"}), ("sdma0", {"HSA_ENABLE_SDMA": "0"})]
for rep in range(2):
  for extra in ([], ["--host-hold", "2600000000"]):
    for name, ev in variants:
      env = {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_SDMA"}
      env.update(ev)
      with open(os.devnull, "wb") as dn:
          t0 = time.perf_counter()
          r = subprocess.run([cli, "--stats"] + extra + [path], stdout=dn, stderr=subprocess.PIPE, env=env)
          dt = time.perf_counter() - t0
      st = json.loads(r.stderr.decode().strip().splitlines()[-1]) if r.returncode == 0 else {}
      print(json.dumps({"variant": name, "extra": extra, "wall_s": round(dt, 4), "rc": r.returncode,
                        **{k: st.get(k) for k in ("create_s", "parse_s", "emit_s", "total_s", "sites_per_s",
                                                   "chunks_held")}}), flush=True)
      if r.returncode:
          print(r.stderr.decode()[-500:])
