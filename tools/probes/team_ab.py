"""A/B of the headline step across libgymsim variants (bench.py's headline leg, several repetitions):
    python tools/probes/team_ab.py libgymsim.so libgymsim_tb32.so"""
import json, os, subprocess, sys
for rep in range(2):
    for lib in sys.argv[1:]:
        env = dict(os.environ, GS_LIBGYMSIM=lib)
        out = subprocess.run([sys.executable, "bench.py", "--steps", "500", "--warmup", "50", "--no-cpu-baseline",
                              "--ppo-epochs", "0", "--other-steps", "0"], env=env, capture_output=True, text=True, timeout=500)
        try:
            d = json.loads(out.stdout.strip().splitlines()[-1])
        except Exception:
            print(lib, "failed", out.stderr[-1500:], flush=True)
            continue
        print(rep, lib, round(d["value"] / 1e6, 3), "M env-steps/s", round(d["ms_per_step"], 4), "ms/step kernel",
              round(d["roofline"]["kernel_ms"], 4), flush=True)
