"""Learning-curve probe: python tools/ppo_probe.py <Task> <epochs> [overrides...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from isaacgymenv_amd.isaacgymenvs import train  # noqa: E402

task, epochs = sys.argv[1], int(sys.argv[2])
t0 = time.time()
agent, stats = train.launch([f"task={task}", "headless=True", f"max_iterations={epochs}",
                             "force_render=False"] + sys.argv[3:], printer=lambda s: print(s, flush=True))
print("done", stats, f"{time.time() - t0:.1f}s", flush=True)
