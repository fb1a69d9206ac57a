"""A/B of the CLI's process exit (SID_EXIT=normal: exit() through the HIP
runtime's teardown; default: _exit after flushing) on the C2 text as a file:
wall clock, start-up (exec to main), the CLI's own clock and the teardown.
Usage: python3 tools/cli_exit_ab.py [sites] [reps]"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import bench
    from sid_amd import gpu as G
    text, ln = G.synth_text_hbm(2, 30.0, 0, n, device=0)
    cli = os.path.join(ROOT, "build", "sid")
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "c2.plp")
        bench.write_text_file(text, ln, path)
        del text
        for rep in range(reps):
            for tag in ("normal", "fast"):
                env = dict(os.environ)
                if tag == "normal":
                    env["SID_EXIT"] = "normal"
                else:
                    env.pop("SID_EXIT", None)
                with open(os.devnull, "wb") as dn:
                    u0 = time.time()
                    r = subprocess.run([cli, "--stats", path], stdout=dn, stderr=subprocess.PIPE, env=env)
                    u1 = time.time()
                st = json.loads(r.stderr.decode().strip().splitlines()[-1])
                print(json.dumps({"tag": tag, "rep": rep, "rc": r.returncode, "wall_s": round(u1 - u0, 4),
                                  "startup_s": round(st["main_entry_unix"] - u0, 4),
                                  "total_s": st["total_s"], "create_s": st["create_s"], "parse_s": st["parse_s"],
                                  "emit_s": st["emit_s"],
                                  "teardown_s": round(u1 - st["main_exit_unix"], 4)}), flush=True)


if __name__ == "__main__":
    main()
