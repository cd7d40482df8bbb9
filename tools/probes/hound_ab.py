"""A/B of the UsefulHound simulate kernel: library variants x self-collision on/off (bench.py's Hound leg).
    python tools/probes/hound_ab.py libgymsim.so:1 libgymsim.so:0 libgymsim_nowave.so:1"""
import json, os, subprocess, sys
for spec in sys.argv[1:]:
    lib, sc = spec.split(":")
    env = dict(os.environ, GS_LIBGYMSIM=lib, GS_SELF_COLLIDE=sc)
    out = subprocess.run([sys.executable, "bench.py", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--ppo-epochs", "0",
                          "--other-steps", "20"], env=env, capture_output=True, text=True, timeout=500)
    try:
        d = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception:
        print(spec, "failed", out.stderr[-2000:], flush=True)
        continue
    print(spec, [(o["task"], round(o["value"] / 1e6, 4), round(o["simulate_kernel_ms"], 4)) for o in d["other_configs"]], flush=True)
