"""UsefulHound simulate kernel alone, for SQ counter passes (tools/probes/hound_sq.sh):
4096 envs, 3 env steps, then 10 gym.simulate launches.  GS_SELF_COLLIDE=0 is the A/B knob."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import isaacgymenvs
    env = isaacgymenvs.make(seed=42, task="UsefulHound", num_envs=int(os.environ.get("N", "4096")), sim_device="cuda:0",
                            rl_device="cuda:0", graphics_device_id=-1, headless=True, force_render=False)
    act = torch.empty((env.num_envs, env.num_actions), device="cuda:0").uniform_(-1, 1)
    env.reset()
    for _ in range(3):
        env.step(act)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(10):
        env.gym.simulate(env.sim)
    ev1.record()
    ev1.synchronize()
    print(f"hound simulate {ev0.elapsed_time(ev1) / 10:.4f} ms/launch, variant {env.gym.amd_kernel_variant(env.sim)}",
          flush=True)


if __name__ == "__main__":
    main()
