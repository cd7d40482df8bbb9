import json, sys, os, subprocess
for lib in ["libgymsim.so", "libgymsim_nl2.so"]:
    env = dict(os.environ, GS_LIBGYMSIM=lib)
    out = subprocess.run([sys.executable, "bench.py", "--steps", "60", "--warmup", "10", "--no-cpu-baseline", "--ppo-epochs", "0"],
                         env=env, capture_output=True, text=True, timeout=400)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    print(lib, [(o["task"], round(o["value"] / 1e6, 3), round(o["simulate_kernel_ms"], 4)) for o in d["other_configs"]], flush=True)
